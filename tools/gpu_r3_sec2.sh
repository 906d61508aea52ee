#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api_device.py tests/test_j2c_sink.py \
  > gpurun_out/r3_generic_tests2.log 2>&1 || { tail -40 gpurun_out/r3_generic_tests2.log; exit 1; }
tail -2 gpurun_out/r3_generic_tests2.log
UDA_DEVICE_REDUCE_TRACE=1 timeout -k 10 600 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 3 --warmup 1 \
  > gpurun_out/r3_bench_api_secondary_48GB_v2.log 2>&1 || { tail -30 gpurun_out/r3_bench_api_secondary_48GB_v2.log; exit 1; }
tail -1 gpurun_out/r3_bench_api_secondary_48GB_v2.log | cut -c1-600
