set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --reducers 16 --steps 3 --warmup 1 > gpurun_out/bench_r16.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --reducers 16 --steps 3 --warmup 1 --sink none > gpurun_out/bench_r16_nosink.log 2>&1 || exit 2
