#!/bin/bash
# Fetch-phase pauses: default vs HIP_ENABLE_DEFERRED_LOADING=0 (all code objects loaded at start-up
# instead of at a kernel's first launch), whole and direct-hybrid variants, 3 repeats each.
set -o pipefail
mkdir -p gpurun_out
for dl in 1 0; do
  HIP_ENABLE_DEFERRED_LOADING=$dl UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py \
    --variants whole,hybrid --repeat 3 > gpurun_out/r3_pause_dl$dl.jsonl 2> gpurun_out/r3_pause_dl$dl.err \
    || { tail -20 gpurun_out/r3_pause_dl$dl.err; exit 1; }
  echo "== HIP_ENABLE_DEFERRED_LOADING=$dl"
  python3 -c "
import json
for line in open('gpurun_out/r3_pause_dl$dl.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'fetch_req_max', (d.get('fetch_req') or {}).get('max_ms'))
"
done
