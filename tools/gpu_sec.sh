set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_decode.py tests/test_properties.py tests/test_gpu_api_device.py > gpurun_out/pt8.log 2>&1 || exit 1
timeout -k 10 200 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec3.log 2>&1 || exit 2
timeout -k 10 300 python benchmarks/run_configs.py netmerger --gb 2 --maps 64 > gpurun_out/nm3.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_sec4 -o run -- python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > /dev/null 2>&1 || exit 4
