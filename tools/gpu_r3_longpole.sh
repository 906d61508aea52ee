#!/bin/bash
# Config #5 (48.5 GB secondary sort through the C ABI, 60 % of every map's records to task 0): the
# skewed task's delivery on a high-priority copy stream (default) vs a normal one, alternating.
set -o pipefail
mkdir -p gpurun_out
for p in 1 0 1 0; do
  log=gpurun_out/r3_longpole_d2h$p.log
  UDA_LONG_POLE_D2H=$p timeout -k 10 600 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 \
    --steps 3 --warmup 1 > $log 2>&1 || { tail -30 $log; exit 1; }
  echo "prio=$p $(grep -o '"value": [0-9.]*\|"validated": [a-z]*' $log | tr '\n' ' ') $(grep -o '"gpu_d2h_wait_ms": [0-9.]*\|"gpu_sink_ms": [0-9.]*\|"total_ms": [0-9.]*' $log | tr '\n' ' ')"
done
