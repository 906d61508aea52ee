cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/r6a/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/r6a/$name.log; [ $rc -le 1 ] || exit $rc; }
step pytest_terasort 420 python -u -m pytest tests/test_gpu_terasort.py -x -v --timeout 150 --timeout-method thread
step stress0 300 python -u tools/multirank_stress.py --steps 40 --out gpurun_out/r6a/stress0.json
step stress24 300 python -u tools/multirank_stress.py --steps 40 --idle-streams 24 --out gpurun_out/r6a/stress24.json
