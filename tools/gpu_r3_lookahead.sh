#!/bin/bash
# k-way lookahead planning A/B (device-only 130 GB) + terasort GPU tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_terasort.py tests/test_gpu_exchange.py \
  > gpurun_out/r3_lookahead_tests.log 2>&1 || { tail -30 gpurun_out/r3_lookahead_tests.log; exit 1; }
tail -2 gpurun_out/r3_lookahead_tests.log
for la in 1 0 1 0; do
  UDA_KWAY_LOOKAHEAD=$la timeout -k 10 300 python -u bench.py --device-only --steps 5 --warmup 1 > gpurun_out/r3_device_only_la$la.log 2>&1 || { tail -20 gpurun_out/r3_device_only_la$la.log; exit 1; }
  echo "lookahead=$la $(tail -1 gpurun_out/r3_device_only_la$la.log | cut -c1-140)"
done
