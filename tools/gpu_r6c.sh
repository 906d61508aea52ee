cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6c
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/r6c/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/r6c/$name.log; [ $rc -le 1 ] || exit $rc; }
step old_memset 300 python -u tools/multirank_stress.py --groups 6 --steps 2 --noise-streams 8 --old-memset 1 --out gpurun_out/r6c/old_memset.json
step fixed_noise 300 python -u tools/multirank_stress.py --groups 10 --steps 4 --noise-streams 8 --out gpurun_out/r6c/fixed_noise.json
export UDA_MULTIRANK_GROUPS=6
step tier 700 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread
