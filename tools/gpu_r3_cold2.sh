#!/bin/bash
# Cold reduce tasks after the prewarm also warms the SDMA engines' queues: host traces, 2 repeats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
UDA_HOST_TRACE=/tmp/cold_tr.csv timeout -k 10 300 python -u tools/cold_task_bench.py --repeat 2 > gpurun_out/r3_cold_trace3.jsonl 2> gpurun_out/r3_cold_trace3.err \
  || { tail -20 gpurun_out/r3_cold_trace3.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r3_cold_trace3.jsonl'):
    d=json.loads(l); t=d.pop('trace',{})
    print(d)
    for k in ('fetch_req','stage_wait','pinned_alloc'):
        v=t.get(k) or {}
        if v.get('n'): print('  ',k,{kk:vv for kk,vv in v.items() if kk not in ('spans_ms','p90_ms')})
    print('   landed', t.get('landed_mb_per_5ms'))
"
