cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6b
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/r6b/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/r6b/$name.log; [ $rc -le 1 ] || exit $rc; }
export UDA_MULTIRANK_GROUPS=6
step tier 700 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread
step noise 300 python -u tools/multirank_stress.py --groups 10 --steps 4 --noise-streams 8 --out gpurun_out/r6b/noise.json
step groups 300 python -u tools/multirank_stress.py --groups 20 --steps 2 --idle-streams 24 --out gpurun_out/r6b/groups.json
