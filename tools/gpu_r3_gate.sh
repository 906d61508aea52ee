#!/bin/bash
# D2H link gate A/B (mapred.uda.gpu.d2h.slots 2 = default vs 0 = ungated): config #5 (C ABI secondary
# sort 48.5 GB, 60 % skew) and 16 concurrent staged tasks over host MOFs (20.8 GB); cold reduce
# tasks with / without the INIT-time prewarm; then the GPU tier.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for sl in 2 0; do
  UDA_API_CONF="mapred.uda.gpu.d2h.slots=$sl" timeout -k 10 400 python -u bench.py --api --workload secondary \
    --rows-per-gpu 470000000 --steps 3 --warmup 1 > gpurun_out/s3e_sec48_slots$sl.log 2>&1 || { tail -30 gpurun_out/s3e_sec48_slots$sl.log; exit 1; }
  echo "== config5 d2h.slots=$sl"; tail -1 gpurun_out/s3e_sec48_slots$sl.log | cut -c1-160
done
for sl in 2 0; do
  UDA_API_CONF="mapred.uda.gpu.d2h.slots=$sl" timeout -k 10 400 python -u bench.py --api --api-host-mofs \
    --rows-per-gpu 200000000 --steps 3 --warmup 1 > gpurun_out/s3e_hostmofs_slots$sl.log 2>&1 || { tail -30 gpurun_out/s3e_hostmofs_slots$sl.log; exit 1; }
  echo "== host MOFs 16 tasks d2h.slots=$sl"; tail -1 gpurun_out/s3e_hostmofs_slots$sl.log | cut -c1-160
done
timeout -k 10 400 python -u tools/cold_task_bench.py --repeat 2 > gpurun_out/r3_cold_tasks.jsonl 2> gpurun_out/r3_cold_tasks.err \
  || { tail -20 gpurun_out/r3_cold_tasks.err; exit 1; }
cat gpurun_out/r3_cold_tasks.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/s3e_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s3e_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s3e_pytest_gpu.log
