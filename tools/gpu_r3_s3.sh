#!/bin/bash
# Round-3 session-3 bundle: GPU tier, J2C threading A/B, direct RPQ vs LPQ hybrid (host traces +
# GenericMerger phase profile of the LPQ variant), config #5 (C ABI secondary sort, 48.5 GB, 60 %
# skew) with the reduce tasks' walker threads vs inline walks, then the flagship bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/s3b_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s3b_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s3b_pytest_gpu.log
timeout -k 10 60 python -u -m pytest -x -q tests/test_j2c_sink.py > gpurun_out/s3b_j2c_tests.log 2>&1 || { tail -20 gpurun_out/s3b_j2c_tests.log; exit 1; }
timeout -k 10 120 python -u tools/j2c_threads_bench.py > gpurun_out/s3b_j2c_threads.txt 2>&1 || { tail -20 gpurun_out/s3b_j2c_threads.txt; exit 1; }
cat gpurun_out/s3b_j2c_threads.txt
UDA_HOST_TRACE=/tmp/uda_tr.csv timeout -k 10 300 python -u tools/netmerger_trace.py --variants whole,hybrid,hybrid_lpq \
  --repeat 3 > gpurun_out/r3_direct_ab.jsonl 2> gpurun_out/r3_direct_ab.err || { tail -20 gpurun_out/r3_direct_ab.err; exit 1; }
python3 -c "
import json
for line in open('gpurun_out/r3_direct_ab.jsonl'):
    d = json.loads(line)
    print(d['variant'], d['gbps'], d['wall_ms'], 'fetch', d.get('fetch_ms'), 'direct', d.get('hybrid_direct'), 'lpqs', d.get('lpqs'), 'rounds', d.get('progressive_rounds'), d['phases_ms'])
"
UDA_GM_PROFILE=1 timeout -k 10 200 python -u tools/netmerger_trace.py --variants hybrid_lpq --repeat 1 \
  > gpurun_out/r3_lpq_gmprof.jsonl 2> gpurun_out/r3_lpq_gmprof.err || { tail -20 gpurun_out/r3_lpq_gmprof.err; exit 1; }
for t in 1 0; do
  UDA_J2C_THREADS=$t timeout -k 10 400 python -u bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 3 --warmup 1 \
    > gpurun_out/s3b_sec48_threads$t.log 2>&1 || { tail -30 gpurun_out/s3b_sec48_threads$t.log; exit 1; }
  echo "== config5 threads=$t"; tail -1 gpurun_out/s3b_sec48_threads$t.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/s3b_bench.log 2>&1 || { tail -30 gpurun_out/s3b_bench.log; exit 1; }
tail -1 gpurun_out/s3b_bench.log | cut -c1-200
