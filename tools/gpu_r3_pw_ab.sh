#!/bin/bash
# Warm-process cost of the INIT prewarm: staged single tasks with / without it (whole-partition and
# progressive), FETCHes right after INIT (no slow-start gap), 3 repeats.
set -o pipefail
mkdir -p gpurun_out
UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,whole_nopw,prog4,prog4_nopw --repeat 3 \
  > gpurun_out/r3_pw_ab.jsonl 2> gpurun_out/r3_pw_ab.err || { tail -20 gpurun_out/r3_pw_ab.err; exit 1; }
python3 -c "
import json
for line in open('gpurun_out/r3_pw_ab.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'prewarm', d.get('prewarm_ms'), 'wait', d.get('prewarm_wait_ms'))
"
