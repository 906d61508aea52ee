cd $GRAFT_REPO_ROOT
python3 tools/gpu_run.py --tag r6f decode_tests pd_tests hybrid41b_s2 hybrid41b_t4 hybrid41b_p16 lzo130x5 lzo130x5_lds pmc_lzo41 pmc_lzo41_lds
