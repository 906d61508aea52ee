#!/bin/bash
# Fetch pauses vs the staging copy engine: whole-partition staged tasks with the early H2D on the SDMA
# engine (default) or as hipMemcpyAsync (UDA_EARLY_H2D_SDMA=0), 4 repeats each in fresh processes.
set -o pipefail
mkdir -p gpurun_out
for e in 1 0; do
  UDA_EARLY_H2D_SDMA=$e UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole --repeat 4 \
    > gpurun_out/r3_pause_sdma$e.jsonl 2> gpurun_out/r3_pause_sdma$e.err || { tail -20 gpurun_out/r3_pause_sdma$e.err; exit 1; }
  echo "== UDA_EARLY_H2D_SDMA=$e"
  python3 -c "
import json
for line in open('gpurun_out/r3_pause_sdma$e.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'req_max', (d.get('fetch_req') or {}).get('max_ms'), 'stage_max', (d.get('stage_wait') or {}).get('max_ms'))
"
done
