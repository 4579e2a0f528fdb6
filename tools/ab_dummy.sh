# A/B: cost of extra empty launches per LM iteration (launch-boundary price) at C4
source tools/gpu_ab.sh
run base MIBA_DUMMY_LAUNCHES=0 && run dummy6 MIBA_DUMMY_LAUNCHES=6 && run dummy12 MIBA_DUMMY_LAUNCHES=12
