#!/bin/bash
# secondary-sort skewed task: per-round trace, single-task baseline, GM phase profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
UDA_DEVICE_REDUCE_TRACE=1 timeout -k 10 300 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 1 --warmup 1 \
  > gpurun_out/r3_sec_trace.log 2>&1 || { tail -30 gpurun_out/r3_sec_trace.log; exit 1; }
grep -c "generic rounds" gpurun_out/r3_sec_trace.log; tail -1 gpurun_out/r3_sec_trace.log | cut -c1-300
UDA_GM_PROFILE=1 timeout -k 10 300 python -u bench.py --api --workload secondary --reducers 1 --rows-per-gpu 280000000 --steps 2 --warmup 1 \
  > gpurun_out/r3_sec_single.log 2>&1 || { tail -30 gpurun_out/r3_sec_single.log; exit 1; }
grep "GM profile" gpurun_out/r3_sec_single.log | tail -3; tail -1 gpurun_out/r3_sec_single.log | cut -c1-300
