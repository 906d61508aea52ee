#!/bin/bash
# Config #5 (C ABI secondary sort, 48.5 GB, 60 % skew) delivery A/B: blit vs SDMA D2H for the generic
# rounds (UDA_NM_D2H_SDMA), with and without the D2H link gate; task 0's wait/sink split per run.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in "0 0" "1 0" "0 2" "1 0" "0 0"; do
  set -- $v
  UDA_NM_D2H_SDMA=$1 UDA_API_CONF="mapred.uda.gpu.d2h.slots=$2" timeout -k 10 400 python -u bench.py --api --workload secondary \
    --rows-per-gpu 470000000 --steps 3 --warmup 1 > gpurun_out/secab_$1_$2.log 2>&1 || { tail -30 gpurun_out/secab_$1_$2.log; exit 1; }
  tail -1 gpurun_out/secab_$1_$2.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); t=d['task0_stats']
print('sdma=$1 slots=$2', d['value'], d['validated'], 'task0 d2h_wait', round(t['gpu_d2h_wait_ms']), 'sink', round(t['gpu_sink_ms']), 'merge', round(t['merge_ms']))"
done
