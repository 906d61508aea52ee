#!/bin/bash
# Cold-task host traces with the registered pinned allocator, then a rocprofv3 kernel-trace profile of
# the flagship step (130 GB, 1 GPU).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
UDA_HOST_TRACE=/tmp/cold_tr.csv timeout -k 10 300 python -u tools/cold_task_bench.py --repeat 1 > gpurun_out/r3_cold_trace2.jsonl 2> gpurun_out/r3_cold_trace2.err \
  || { tail -20 gpurun_out/r3_cold_trace2.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r3_cold_trace2.jsonl'):
    d=json.loads(l); t=d.pop('trace',{})
    print(d)
    for k in ('fetch_req','stage_wait','pinned_alloc','pinned_buf_alloc'):
        v=t.get(k) or {}
        if v.get('n'): print('  ',k,{kk:vv for kk,vv in v.items() if kk!='spans_ms'}, (v.get('spans_ms') or [])[:10])
    print('   landed', t.get('landed_mb_per_5ms'))
"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 3 --warmup 1 \
  > gpurun_out/r3_final_prof_bench.log 2>&1 || { tail -30 gpurun_out/r3_final_prof_bench.log; exit 1; }
tail -1 gpurun_out/r3_final_prof_bench.log | cut -c1-160
find gpurun_out/prof_final -name "*stats*" | head
