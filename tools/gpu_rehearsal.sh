set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python tools/local_group_rehearsal.py --world 8 --rows-per-rank 20000000 > gpurun_out/rehearsal8.log 2>&1 || exit 1
