set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S="python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcS_a -o run -- $S > /dev/null 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pmcS_d -o run -- $S > /dev/null 2>&1 || exit 4
