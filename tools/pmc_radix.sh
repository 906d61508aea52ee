# PMC passes over the F8 map-side radix sort (benchmarks/run_configs.py radix): one run per counter group.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
S="python benchmarks/run_configs.py radix --gb 0.8"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc1_radix -o run -- $S > gpurun_out/pmc_radix1.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc2_radix -o run -- $S > gpurun_out/pmc_radix2.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc3_radix -o run -- $S > gpurun_out/pmc_radix3.log 2>&1 || exit 5
python tools/pmc_summary.py gpurun_out/pmc1_radix gpurun_out/pmc2_radix gpurun_out/pmc3_radix > gpurun_out/pmc_radix_summary.md
