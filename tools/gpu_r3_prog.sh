#!/bin/bash
# Progressive NetMerger phases: correctness (GPU consumer tests), then the 2 GB single-task secondary
# sort over host MOFs with the host-event trace: whole-partition staging vs 2/4/8 progressive phases.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generic.py \
  -k "consumer or progressive" > gpurun_out/r3_prog_tests.log 2>&1 || { tail -40 gpurun_out/r3_prog_tests.log; exit 1; }
tail -1 gpurun_out/r3_prog_tests.log
UDA_HOST_TRACE=/tmp/uda_trace_$$.csv timeout -k 10 400 python -u tools/netmerger_trace.py --variants whole,prog2,prog4,prog8 \
  > gpurun_out/r3_prog_trace.jsonl 2> gpurun_out/r3_prog_trace.err || { tail -20 gpurun_out/r3_prog_trace.err; exit 1; }
cut -c1-220 gpurun_out/r3_prog_trace.jsonl
