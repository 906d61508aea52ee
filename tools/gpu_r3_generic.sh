#!/bin/bash
# Round 3: generic key-range rounds + secondary-sort C-ABI bench at scale.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_api_device.py \
  tests/test_properties.py tests/test_gpu_generic.py > gpurun_out/r3_generic_tests.log 2>&1 || { tail -40 gpurun_out/r3_generic_tests.log; exit 1; }
tail -3 gpurun_out/r3_generic_tests.log
timeout -k 10 600 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 3 --warmup 1 \
  > gpurun_out/r3_bench_api_secondary_50GB.log 2>&1 || { tail -30 gpurun_out/r3_bench_api_secondary_50GB.log; exit 1; }
tail -1 gpurun_out/r3_bench_api_secondary_50GB.log
