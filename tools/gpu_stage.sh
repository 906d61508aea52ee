set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
{ cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null; nproc; } > gpurun_out/cg_before.txt 2>&1
export UDA_STAGE_TRACE=1
timeout -k 10 300 python benchmarks/run_configs.py netmerger --gb 2 --maps 64 --reducers 1 > gpurun_out/st_drains.log 2>&1 || exit 1
cat /sys/fs/cgroup/cpu.stat > gpurun_out/cg_after.txt 2>&1 || true
