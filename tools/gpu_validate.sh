#!/bin/bash
# One GPU-box validation pass: the GPU test tier, then the default 1-GPU headline bench.
# Usage (from the dev container): gpurun --timeout 900 -- 'bash tools/gpu_validate.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 360 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_default.json \
    2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
