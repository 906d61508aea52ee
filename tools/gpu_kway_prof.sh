set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_terasort.py > gpurun_out/pt10.log 2>&1 || exit 1
S="python bench.py --device-only --rows-per-gpu 100000000 --steps 1 --warmup 1 --no-validate"
B="python bench.py --device-only --steps 3 --warmup 1"
for cap in 1536 1024; do
  UDA_KWAY_PROF=1 UDA_KWAY_CAP=$cap timeout -k 10 200 $S > gpurun_out/prof_$cap.log 2>&1 || exit 2
  UDA_KWAY_CAP=$cap timeout -k 10 200 $B > gpurun_out/cap_$cap.log 2>&1 || exit 3
done
