# Round profile set (run on the GPU box from the repo root): bench lines C2/C4/C5, rocprofv3 kernel
# trace + stats of the C4 bench, and two PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic.
# Outputs under gpurun_out/prof/; summarised into profiles/ by tools/prof_summary.py / pmc_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_c4.log 2>&1 || { echo BENCH_C4_FAIL; tail -5 $O/bench_c4.log; exit 1; }
timeout -k 10 200 python bench.py --config C2 --no-cpu-baseline > $O/bench_c2.log 2>&1 || { echo BENCH_C2_FAIL; exit 1; }
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --steps 10 > $O/bench_c5.log 2>&1 || { echo BENCH_C5_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 20 --no-profile --no-cpu-baseline > $O/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o f -- python3 bench.py --steps 10 --warmup 1 --no-profile --no-cpu-baseline > $O/pmc_f.log 2>&1 || { echo PMC_F_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o w -- python3 bench.py --steps 10 --warmup 1 --no-profile --no-cpu-baseline > $O/pmc_w.log 2>&1 || { echo PMC_W_FAIL; exit 1; }
echo PROFILE_OK
