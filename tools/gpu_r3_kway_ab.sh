#!/bin/bash
# k-way merge A/B: non-temporal F4 stores on/off, device-only (merge alone), 130 GB
set -o pipefail
mkdir -p gpurun_out
for nt in 1 0 1 0; do
  UDA_KWAY_NT=$nt timeout -k 10 300 python -u bench.py --device-only --steps 5 --warmup 1 --no-validate > gpurun_out/r3_kway_nt$nt.log 2>&1 || { tail -20 gpurun_out/r3_kway_nt$nt.log; exit 1; }
  echo "nt=$nt $(tail -1 gpurun_out/r3_kway_nt$nt.log | cut -c1-160)"
done
