set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 tools/rccl_shared_gpu.py > gpurun_out/rccl2_zc.log 2>&1 || exit 1
UDA_RCCL_PACK=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 tools/rccl_shared_gpu.py > gpurun_out/rccl2_pack.log 2>&1 || exit 2
