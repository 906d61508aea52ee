#!/bin/bash
# k-way merge A/B: in-place LDS merge (one buffer per workgroup, more workgroups per CU) vs two buffers,
# at several cell capacities; device-only (merge alone), 130 GB. Correctness first.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_terasort.py \
  -k "kway" > gpurun_out/r3_inplace_tests.log 2>&1 || { tail -30 gpurun_out/r3_inplace_tests.log; exit 1; }
tail -1 gpurun_out/r3_inplace_tests.log
for cfg in "0 1536" "1 1536" "1 2048" "1 1024" "1 1536"; do
  set -- $cfg
  log=gpurun_out/r3_kway_inplace$1_cap$2.log
  UDA_KWAY_INPLACE=$1 UDA_KWAY_CAP=$2 timeout -k 10 300 python -u bench.py --device-only --steps 5 --warmup 1 --no-validate \
    > $log 2>&1 || { tail -20 $log; exit 1; }
  echo "inplace=$1 cap=$2 $(tail -1 $log | cut -c1-140)"
done
