cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6d
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/r6d/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/r6d/$name.log | cut -c1-400; [ $rc -le 1 ] || exit $rc; }
step old2 300 python -u tools/multirank_stress.py --groups 10 --steps 4 --noise-streams 8 --old-memset 2 --out gpurun_out/r6d/old2.json
step old1 300 python -u tools/multirank_stress.py --groups 10 --steps 4 --noise-streams 8 --old-memset 1 --out gpurun_out/r6d/old1.json
step new 300 python -u tools/multirank_stress.py --groups 10 --steps 4 --noise-streams 8 --out gpurun_out/r6d/new.json
