set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_api_device.py > gpurun_out/gen_tests.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec_new.log 2>&1 || exit 2
UDA_F2_SEPARATE=1 timeout -k 10 300 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec_f2sep.log 2>&1 || exit 3
UDA_GATHER_LANES=4 timeout -k 10 300 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec_g4.log 2>&1 || exit 4
timeout -k 10 300 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec_new2.log 2>&1 || exit 5
