set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S="python bench.py --device-only --rows-per-gpu 100000000 --steps 1 --warmup 0 --no-validate"
for cap in 1536 1024; do
  export UDA_KWAY_CAP=$cap
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcA_$cap -o run -- $S > /dev/null 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcB_$cap -o run -- $S > /dev/null 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcC_$cap -o run -- $S > /dev/null 2>&1 || exit 5
done
