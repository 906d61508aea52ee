#!/bin/bash
# Round 3: C-ABI path after pooling the per-task device-merge workspaces.
set -o pipefail
mkdir -p gpurun_out /tmp/udamof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api_device.py \
  > gpurun_out/r3_api_tests.log 2>&1 || { tail -40 gpurun_out/r3_api_tests.log; exit 1; }
tail -2 gpurun_out/r3_api_tests.log
for mode in reg files; do
  extra=""; [ $mode = files ] && extra="--mof-dir /tmp/udamof"
  timeout -k 10 600 python -u bench.py --api $extra --rows-per-gpu 400000000 --steps 3 --warmup 1 \
    > gpurun_out/r3_bench_api_${mode}_41GB.log 2>&1 || { tail -30 gpurun_out/r3_bench_api_${mode}_41GB.log; exit 1; }
  tail -1 gpurun_out/r3_bench_api_${mode}_41GB.log | cut -c1-400
done
timeout -k 10 600 python -u bench.py --api --steps 3 --warmup 1 > gpurun_out/r3_bench_api_130GB.log 2>&1 || { tail -30 gpurun_out/r3_bench_api_130GB.log; exit 1; }
tail -1 gpurun_out/r3_bench_api_130GB.log | cut -c1-400
