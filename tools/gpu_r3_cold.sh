#!/bin/bash
# Cold reduce tasks (one process each, INIT, 1 s slow-start gap, 64 FETCHes): INIT-time GPU prewarm
# on vs off; then the GPU tier.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/cold_task_bench.py --repeat 2 > gpurun_out/r3_cold_tasks.jsonl 2> gpurun_out/r3_cold_tasks.err \
  || { tail -20 gpurun_out/r3_cold_tasks.err; exit 1; }
cat gpurun_out/r3_cold_tasks.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/s3d_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s3d_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s3d_pytest_gpu.log
