#!/bin/bash
# Progressive NetMerger phases (tests + trace), vectorized F6 decode (tests + compressed C-ABI benches),
# in-place k-way A/B (tools/gpu_r3_inplace.sh).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_r3_prog.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_decode.py \
  tests/test_gpu_api_device.py -k "decode or codec or compress or snappy or lzo" > gpurun_out/r3_decode_tests.log 2>&1 \
  || { tail -30 gpurun_out/r3_decode_tests.log; exit 1; }
tail -1 gpurun_out/r3_decode_tests.log
for c in snappy lzo; do
  timeout -k 10 600 python -u bench.py --api --api-codec $c --rows-per-gpu 400000000 --steps 3 --warmup 1 \
    > gpurun_out/r3_bench_api_${c}_41GB_vec.log 2>&1 || { tail -20 gpurun_out/r3_bench_api_${c}_41GB_vec.log; exit 1; }
  echo "$c $(tail -1 gpurun_out/r3_bench_api_${c}_41GB_vec.log | cut -c1-150)"
done
bash tools/gpu_r3_inplace.sh || exit 1
