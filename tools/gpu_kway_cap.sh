set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_terasort.py > gpurun_out/pt9.log 2>&1 || exit 1
B="python bench.py --device-only --steps 3 --warmup 1 --no-validate"
for cap in 2048 1536 1024; do
  UDA_KWAY_CAP=$cap timeout -k 10 200 $B > gpurun_out/cap_$cap.log 2>&1 || exit 2
done
timeout -k 10 200 python bench.py --device-only --steps 3 --warmup 1 > gpurun_out/cap_validated.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="python bench.py --device-only --rows-per-gpu 100000000 --steps 1 --warmup 0 --no-validate"
for cap in 1536 1024; do
  UDA_KWAY_CAP=$cap timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_cap$cap -o run -- $S > /dev/null 2>&1 || exit 4
done
