#!/bin/bash
# Pinned host memory from registered THP-backed pages (sdma.h pinned_host_alloc): GPU tier, cold reduce
# tasks, the staged NetMerger variants, the 16-task host-MOF C-ABI bench and the flagship bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/s3f_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s3f_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s3f_pytest_gpu.log
timeout -k 10 300 python -u tools/cold_task_bench.py --repeat 2 > gpurun_out/r3_cold_tasks2.jsonl 2> gpurun_out/r3_cold_tasks2.err \
  || { tail -20 gpurun_out/r3_cold_tasks2.err; exit 1; }
cat gpurun_out/r3_cold_tasks2.jsonl
UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,hybrid --repeat 2 \
  > gpurun_out/r3_nm_pinned.jsonl 2> gpurun_out/r3_nm_pinned.err || { tail -20 gpurun_out/r3_nm_pinned.err; exit 1; }
python3 -c "
import json
for line in open('gpurun_out/r3_nm_pinned.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'pinned_alloc', (d.get('pinned_alloc') or {}).get('sum_ms'))
"
timeout -k 10 400 python -u bench.py --api --api-host-mofs --rows-per-gpu 200000000 --steps 3 --warmup 1 > gpurun_out/s3f_hostmofs.log 2>&1 \
  || { tail -30 gpurun_out/s3f_hostmofs.log; exit 1; }
echo "== host MOFs 16 tasks"; tail -1 gpurun_out/s3f_hostmofs.log | cut -c1-160
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/s3f_bench.log 2>&1 || { tail -30 gpurun_out/s3f_bench.log; exit 1; }
echo "== flagship"; tail -1 gpurun_out/s3f_bench.log | cut -c1-160
grep "^# setup" gpurun_out/s3f_bench.log | cut -c1-200
