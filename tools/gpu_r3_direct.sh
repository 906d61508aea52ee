#!/bin/bash
# Direct RPQ vs the LPQ level on the DRAM tier (2 GB secondary sort, one task, budget = input / 6):
# hybrid/consumer tests, then host-event traces of both (index, per-round H2D / merge / delivery spans).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generic.py \
  -k "hybrid or consumer" > gpurun_out/r3_direct_tests.log 2>&1 || { tail -30 gpurun_out/r3_direct_tests.log; exit 1; }
tail -1 gpurun_out/r3_direct_tests.log
UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,hybrid,hybrid_lpq \
  --repeat 3 > gpurun_out/r3_direct_ab.jsonl 2> gpurun_out/r3_direct_ab.err || { tail -20 gpurun_out/r3_direct_ab.err; exit 1; }
python3 -c "
import json
for line in open('gpurun_out/r3_direct_ab.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'direct', d.get('hybrid_direct'), 'lpqs', d.get('lpqs'), 'rounds', d.get('progressive_rounds'), d['phases_ms'])
    print('    vm', d.get('vm_deltas'))
    for k in ('index', 'dm_h2d', 'dm_merge', 'rpq_deliver'):
        v = d.get(k)
        if v and v.get('n'):
            print('   ', k, {kk: vv for kk, vv in v.items() if kk != 'spans_ms'}, (v.get('spans_ms') or [])[:14])
"
