cd $GRAFT_REPO_ROOT
bash tools/gpu_r6d.sh || exit $?
python3 tools/gpu_run.py --tag r6e decode_tests pd_tests hybrid41b_s2 hybrid41b_noprog lzo130x5
