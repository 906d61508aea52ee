#!/bin/bash
# GPU tier after the merger/decoder allocation changes, the direct-RPQ trace, and the C-ABI
# compressed (LZO) and host-MOF 16-task benches that run many concurrent generic merges / decodes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/s3c_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s3c_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s3c_pytest_gpu.log
bash tools/gpu_r3_direct.sh || exit 1
timeout -k 10 400 python -u bench.py --api --api-codec lzo --rows-per-gpu 400000000 --steps 3 --warmup 1 > gpurun_out/s3c_api_lzo.log 2>&1 || { tail -30 gpurun_out/s3c_api_lzo.log; exit 1; }
echo "== api lzo"; tail -1 gpurun_out/s3c_api_lzo.log | cut -c1-200
