#!/bin/bash
# Where the 50-95 ms stalls of the staged NetMerger path come from: host trace with pinned/device
# allocation events, whole vs hybrid, three repeats.
set -o pipefail
mkdir -p gpurun_out
UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,hybrid --repeat 3 \
  > gpurun_out/r3_hybrid_alloc.jsonl 2> gpurun_out/r3_hybrid_alloc.err || { tail -20 gpurun_out/r3_hybrid_alloc.err; exit 1; }
python3 -c "
import json
for line in open('gpurun_out/r3_hybrid_alloc.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'))
    for k in ('lpq_merge', 'stage_wait', 'drain', 'pinned_alloc', 'device_alloc', 'device_free'):
        v = d.get(k)
        if v and v.get('n'):
            print('   ', k, {kk: vv for kk, vv in v.items() if kk != 'spans_ms'}, (v.get('spans_ms') or [])[:8])
"
