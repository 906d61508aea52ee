set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_api_device.py > gpurun_out/gen_tests.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec_new.log 2>&1 || exit 2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/secprof2 -o run -- python3 $R/benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > $R/gpurun_out/sec_prof.log 2>&1 || exit 3
