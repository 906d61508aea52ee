set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_final -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/kt_final.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcG_a -o run -- python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > /dev/null 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcG_b -o run -- python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > /dev/null 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcG_c -o run -- python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > /dev/null 2>&1 || exit 4
