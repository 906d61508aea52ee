set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/udad
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_terasort.py -k "spill or disk" > gpurun_out/pt14.log 2>&1 || exit 1
UDA_ROUND_TRACE=1 timeout -k 10 500 python bench.py --store disk --local-dirs /tmp/udad --rows-per-gpu 600000000 --steps 1 --warmup 1 --max-round-gb 4 > gpurun_out/disk_stage.log 2>&1 || exit 2
rm -rf /tmp/udad
