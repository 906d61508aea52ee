#!/bin/bash
# Progressive NetMerger phases under 16 concurrent reduce tasks: C-ABI bench with host-resident MOFs
# (20.8 GB, 6 admitted GPU merges), mapred.uda.gpu.progressive.phases 0 vs 4, alternating.
set -o pipefail
mkdir -p gpurun_out
for ph in 0 4 0 4; do
  log=gpurun_out/r3_api_host_prog$ph.log
  UDA_API_CONF="mapred.uda.gpu.progressive.phases=$ph" timeout -k 10 300 python -u bench.py --api --api-host-mofs \
    --rows-per-gpu 200000000 --steps 3 --warmup 1 > $log 2>&1 || { tail -20 $log; exit 1; }
  echo "phases=$ph $(grep -o '"value": [0-9.]*\|"validated": [a-z]*' $log | tr '\n' ' ')"
done
