#!/bin/bash
# k-way merge configuration sweep, device-only (merge alone), 130 GB: in-place LDS merge (5 workgroups
# per CU instead of 3), cell capacity, target fill of a cell (UDA_KWAY_FILL, % of the capacity; the rest
# is the sampling slack) and F3 outputs spread over all threads (UDA_KWAY_SPREAD). Correctness first.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_terasort.py \
  -k "kway" > gpurun_out/r3_kway_cfg_tests.log 2>&1 || { tail -30 gpurun_out/r3_kway_cfg_tests.log; exit 1; }
tail -1 gpurun_out/r3_kway_cfg_tests.log
i=0
for cfg in "${@:-INPLACE=0,CAP=1536,FILL=50 INPLACE=1,CAP=1536,FILL=50 INPLACE=0,CAP=1536,FILL=50,SPREAD=1 INPLACE=1,CAP=1536,FILL=50,SPREAD=1 INPLACE=1,CAP=1536,FILL=70 INPLACE=1,CAP=1024,FILL=60,SPREAD=1 INPLACE=1,CAP=2048,FILL=50,SPREAD=1 INPLACE=0,CAP=1536,FILL=50}"; do
  for c in $cfg; do
    i=$((i+1))
    envs=$(echo $c | tr ',' ' ' | sed 's/\([A-Z]*=\)/UDA_KWAY_\1/g')
    log=gpurun_out/r3_kway_cfg$i.log
    env $envs timeout -k 10 300 python -u bench.py --device-only --steps 5 --warmup 1 --no-validate > $log 2>&1 \
      || { tail -20 $log; exit 1; }
    echo "$c $(tail -1 $log | cut -c1-140)"
  done
done
