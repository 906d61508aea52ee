#!/bin/bash
# Round 3 batch: lookahead A/B + terasort/exchange tests, compressed C-ABI benches, SDMA delivery A/B
# for the skewed secondary sort, full GPU tier.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_r3_lookahead.sh || exit 1
for c in snappy lzo; do
  timeout -k 10 600 python -u bench.py --api --api-codec $c --rows-per-gpu 400000000 --steps 3 --warmup 1 \
    > gpurun_out/r3_bench_api_${c}_41GB.log 2>&1 || { tail -20 gpurun_out/r3_bench_api_${c}_41GB.log; exit 1; }
  echo "$c $(tail -1 gpurun_out/r3_bench_api_${c}_41GB.log | cut -c1-150)"
done
for v in 1 0; do
  UDA_NM_D2H_SDMA=$v timeout -k 10 300 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 3 --warmup 1 \
    > gpurun_out/r3_sec_sdma$v.log 2>&1 || { tail -20 gpurun_out/r3_sec_sdma$v.log; exit 1; }
  echo "sdma=$v $(tail -1 gpurun_out/r3_sec_sdma$v.log | cut -c1-120)"
done
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3_pytest_gpu_full2.log 2>&1 || { tail -30 gpurun_out/r3_pytest_gpu_full2.log; exit 1; }
tail -2 gpurun_out/r3_pytest_gpu_full2.log
