#!/bin/bash
# Round 3: provider HBM store + descriptor fallbacks + checkpoint/device-path tests, then --api --mof-dir at scale.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_api_device.py tests/test_gpu_generic.py > gpurun_out/r3_provider_tests.log 2>&1 || { tail -40 gpurun_out/r3_provider_tests.log; exit 1; }
tail -3 gpurun_out/r3_provider_tests.log
mkdir -p /tmp/udamof
timeout -k 10 600 python -u bench.py --api --mof-dir /tmp/udamof --rows-per-gpu 400000000 --steps 3 --warmup 1 \
  > gpurun_out/r3_bench_api_mof_files.log 2>&1 || { tail -30 gpurun_out/r3_bench_api_mof_files.log; exit 1; }
tail -1 gpurun_out/r3_bench_api_mof_files.log
