cd $GRAFT_REPO_ROOT
MIBA_SCHUR_STAMPS=1 timeout -k 10 120 python tools/kernel_stamps.py C4 1 > gpurun_out/schur_stamps_c4.log 2>&1 || echo STAMPS_FAIL
