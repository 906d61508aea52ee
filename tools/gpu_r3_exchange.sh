#!/bin/bash
# Round 3: exchange backends + multi-process shuffle on the one-GPU box.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_exchange.py tests/test_gpu_terasort.py > gpurun_out/r3_exchange_tests.log 2>&1 || { tail -40 gpurun_out/r3_exchange_tests.log; exit 1; }
tail -5 gpurun_out/r3_exchange_tests.log
# multi-process rehearsal at scale: 2 and 4 rank processes on GPU 0 (ipc exchange)
timeout -k 10 400 python -u bench.py --gpus 2 --one-gpu --exchange ipc --rows-per-gpu 300000000 --steps 3 --warmup 1 \
  > gpurun_out/r3_bench_ipc_2ranks.log 2>&1 || { tail -30 gpurun_out/r3_bench_ipc_2ranks.log; exit 1; }
tail -3 gpurun_out/r3_bench_ipc_2ranks.log
timeout -k 10 400 python -u bench.py --gpus 4 --one-gpu --exchange ipc --rows-per-gpu 150000000 --steps 3 --warmup 1 \
  > gpurun_out/r3_bench_ipc_4ranks.log 2>&1 || { tail -30 gpurun_out/r3_bench_ipc_4ranks.log; exit 1; }
tail -3 gpurun_out/r3_bench_ipc_4ranks.log
