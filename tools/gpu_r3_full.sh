#!/bin/bash
# Round 3: full GPU tier, then the multi-process rehearsal benches (ipc exchange, ranks on GPU 0).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3_pytest_gpu.log
for n in 2 4; do
  rows=$((600000000 / n))
  timeout -k 10 400 python -u bench.py --gpus $n --one-gpu --exchange ipc --rows-per-gpu $rows --steps 3 --warmup 1 \
    > gpurun_out/r3_bench_ipc_${n}ranks.log 2>&1 || { tail -30 gpurun_out/r3_bench_ipc_${n}ranks.log; exit 1; }
  tail -1 gpurun_out/r3_bench_ipc_${n}ranks.log
done
