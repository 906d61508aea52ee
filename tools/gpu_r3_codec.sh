#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_api_device.py tests/test_gpu_decode.py tests/test_gpu_generic.py \
  > gpurun_out/r3_codec_tests.log 2>&1 || { tail -40 gpurun_out/r3_codec_tests.log; exit 1; }
tail -3 gpurun_out/r3_codec_tests.log
bash tools/gpu_r3_sec2.sh
bash tools/gpu_r3_kway_ab.sh
