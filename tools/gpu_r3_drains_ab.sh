#!/bin/bash
# 16 staged tasks over host MOFs (C ABI, 20.8 GB, 6 merge slots): drain threads per task 8 (default) / 4 / 2.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for d in 8 4 2 8; do
  UDA_API_CONF="mapred.uda.gpu.fetch.drains=$d" timeout -k 10 300 python -u bench.py --api --api-host-mofs \
    --rows-per-gpu 200000000 --steps 3 --warmup 1 > gpurun_out/drains_$d.log 2>&1 || { tail -30 gpurun_out/drains_$d.log; exit 1; }
  echo "drains=$d $(tail -1 gpurun_out/drains_$d.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["validated"])')"
done
