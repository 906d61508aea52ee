set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --device-only --steps 3 --warmup 1 --no-validate"
timeout -k 10 200 $B > gpurun_out/dev_kway.log 2>&1 || exit 1
UDA_KWAY=0 timeout -k 10 200 $B > gpurun_out/dev_tree.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="python bench.py --device-only --rows-per-gpu 100000000 --steps 1 --warmup 0 --no-validate"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_kway -o run -- $S > /dev/null 2>&1 || exit 2
for mode in kway tree; do
  if [ $mode = tree ]; then export UDA_KWAY=0; else unset UDA_KWAY; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc1_$mode -o run -- $S > /dev/null 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc2_$mode -o run -- $S > /dev/null 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc3_$mode -o run -- $S > /dev/null 2>&1 || exit 5
done
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_api_device.py > gpurun_out/pt7.log 2>&1 || exit 6
timeout -k 10 200 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec2.log 2>&1 || exit 7
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_sec -o run -- python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > /dev/null 2>&1 || exit 8
