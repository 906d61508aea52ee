#!/bin/bash
# K-way merge evidence with the round-3 defaults: kernel trace of the full 130 GB device-only step
# (kernel time vs planning vs gaps), then PMC passes on a 100M-row step (one pass per counter group).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3kt -o run -- \
  python3 bench.py --device-only --steps 2 --warmup 1 --no-validate > gpurun_out/r3kt.log 2>&1 || { tail -5 gpurun_out/r3kt.log; exit 1; }
S="python3 bench.py --device-only --rows-per-gpu 100000000 --steps 1 --warmup 0 --no-validate"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/r3pmcA -o run -- $S > /dev/null 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3pmcB -o run -- $S > /dev/null 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r3pmcC -o run -- $S > /dev/null 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d gpurun_out/r3pmcD -o run -- $S > /dev/null 2>&1 || exit 6
python3 tools/pmc_summary.py gpurun_out/r3pmcA gpurun_out/r3pmcB gpurun_out/r3pmcC > gpurun_out/r3pmc_summary.txt 2>&1
echo done
