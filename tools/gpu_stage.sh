set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export UDA_STAGE_TRACE=1
timeout -k 10 300 python benchmarks/run_configs.py netmerger --gb 2 --maps 64 --reducers 1 > gpurun_out/st_sdma.log 2>&1 || exit 1
UDA_EARLY_H2D_SDMA=0 timeout -k 10 300 python benchmarks/run_configs.py netmerger --gb 2 --maps 64 --reducers 1 > gpurun_out/st_hip.log 2>&1 || exit 2
