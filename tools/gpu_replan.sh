set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_terasort.py -k replan > gpurun_out/replan_tests.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_noreplan.log 2>&1 || exit 2
timeout -k 10 500 python bench.py --steps 3 --warmup 1 --replan > gpurun_out/bench_replan.log 2>&1 || exit 3
