set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_terasort.py -k "spill or disk" > gpurun_out/pt14.log 2>&1 || exit 1
B="python bench.py --store host --rows-per-gpu 600000000 --steps 2 --warmup 1 --max-round-gb 4"
UDA_ROUND_TRACE=1 timeout -k 10 300 $B > gpurun_out/sp_trace.log 2>&1 || exit 2
