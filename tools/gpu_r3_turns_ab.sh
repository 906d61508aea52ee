#!/bin/bash
# Config #5 (C ABI secondary sort 48.5 GB, 60 % skew): generic device merges taking turns
# (mapred.uda.gpu.merge.slots, the next turn to the task with the most input left) vs all at once.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for ms in 0 1 2 4 0 1; do
  UDA_API_CONF="mapred.uda.gpu.merge.slots=$ms" timeout -k 10 400 python -u bench.py --api --workload secondary \
    --rows-per-gpu 470000000 --steps 3 --warmup 1 > gpurun_out/turns_$ms.log 2>&1 || { tail -30 gpurun_out/turns_$ms.log; exit 1; }
  tail -1 gpurun_out/turns_$ms.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); t=d['task0_stats']
print('merge.slots=$ms', d['value'], d['validated'], 'task0 merge', round(t['merge_ms']), 'd2h_wait', round(t['gpu_d2h_wait_ms']), 'sink', round(t['gpu_sink_ms']))"
done
