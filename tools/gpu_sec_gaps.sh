set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > gpurun_out/sec_warm.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/secprof -o run -- python3 $R/benchmarks/run_configs.py secondary_sort --gb 2 --maps 64 > $R/gpurun_out/sec_prof.log 2>&1 || exit 2
