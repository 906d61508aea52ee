#!/bin/bash
# W > 1 spill tiers: 2 real processes on GPU 0 over the IPC exchange, staging on the SDMA thread
set -o pipefail
mkdir -p gpurun_out
for st in host disk; do
  rows=200000000; [ $st = disk ] && rows=100000000
  log=gpurun_out/r3_bench_ipc2_store_$st.log
  timeout -k 10 600 python -u bench.py --gpus 2 --one-gpu --exchange ipc --store $st --rows-per-gpu $rows --steps 3 --warmup 1 \
    > $log 2>&1 || { tail -20 $log; exit 1; }
  echo "store=$st $(tail -1 $log | cut -c1-200)"
done
