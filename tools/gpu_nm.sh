set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_api_device.py tests/test_gpu_decode.py > gpurun_out/nm_tests.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/run_configs.py netmerger --gb 2 --maps 64 --reducers 4 > gpurun_out/nm4.log 2>&1 || exit 2
