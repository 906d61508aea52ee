#!/bin/bash
# GPU hybrid merge (LPQ spills to pinned DRAM, RPQ key-range rounds), one 2 GB secondary-sort task:
# hybrid tests, then the host-event trace with LPQ spill D2H / RPQ H2D on SDMA engines (default) vs
# blit kernels, with the cgroup CPU-throttle deltas per variant.
set -o pipefail
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max > gpurun_out/cpu_max.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generic.py \
  -k "hybrid or consumer" > gpurun_out/r3_hyb_tests.log 2>&1 || { tail -30 gpurun_out/r3_hyb_tests.log; exit 1; }
tail -1 gpurun_out/r3_hyb_tests.log
i=0
for envs in "X=1" "UDA_RPQ_H2D_SDMA=0 UDA_LPQ_D2H_SDMA=0" "UDA_RPQ_H2D_SDMA=0" "UDA_LPQ_D2H_SDMA=0"; do
  i=$((i+1))
  env $envs UDA_HOST_TRACE=/tmp/uda_tr_$i.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,hybrid \
    --repeat 3 > gpurun_out/r3_hybrid_ab$i.jsonl 2> gpurun_out/r3_hybrid_ab$i.err || { tail -20 gpurun_out/r3_hybrid_ab$i.err; exit 1; }
  echo "== $envs"
  python3 -c "
import json
for line in open('gpurun_out/r3_hybrid_ab$i.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'thr', d.get('cpu_throttled'), d['phases_ms'])
"
done
