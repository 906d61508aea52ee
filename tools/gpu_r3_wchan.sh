#!/bin/bash
# Where the 40-75 ms process-wide pauses of the staged NetMerger fetch sit: per-thread kernel wait
# channels sampled every ~2 ms through each task (whole and direct-hybrid variants).
set -o pipefail
mkdir -p gpurun_out
UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,hybrid --repeat 3 --wchan \
  > gpurun_out/r3_wchan.jsonl 2> gpurun_out/r3_wchan.err || { tail -20 gpurun_out/r3_wchan.err; exit 1; }
python3 -c "
import json
for line in open('gpurun_out/r3_wchan.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], 'fetch_req_max', (d.get('fetch_req') or {}).get('max_ms'), 'landed', d.get('landed_mb_per_5ms'))
    w = d.get('wchan') or {}
    print('   ', w.get('busy_waits'))
    print('    futex', w.get('contended_futex'))
    for k in ('pinned_alloc', 'pinned_buf_alloc', 'device_alloc', 'device_free'):
        v = d.get(k) or {}
        if v.get('n'):
            print('   ', k, v.get('n'), v.get('sum_ms'), (v.get('spans_ms') or [])[:8])
"
