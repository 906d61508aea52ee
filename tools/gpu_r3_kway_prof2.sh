#!/bin/bash
# per-phase K-way timings (UDA_KWAY_PROF, 100M rows) for the given env combos (same syntax as gpu_r3_kway_cfg.sh)
set -o pipefail
mkdir -p gpurun_out
i=0
for c in "$@"; do
  i=$((i+1))
  envs=$(echo $c | tr ',' ' ' | sed 's/\([A-Z]*=\)/UDA_KWAY_\1/g')
  log=gpurun_out/r3_kway_prof$i.log
  env UDA_KWAY_PROF=1 $envs timeout -k 10 200 python -u bench.py --device-only --rows-per-gpu 100000000 --steps 1 \
    --warmup 1 --no-validate > $log 2>&1 || { tail -20 $log; exit 1; }
  echo "$c $(grep 'kway phases' $log | tail -1)"
done
