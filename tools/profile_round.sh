# Round profile set (run on the GPU box from the repo root): bench lines C1-C5, rocprofv3 kernel traces + stats of
# the C4 and C5 benches, two PMC passes (FETCH_SIZE, WRITE_SIZE) and one SQ pass on C4, and the BCR / band-tail stamp
# timelines. Outputs under gpurun_out/prof/; summarised into profiles/ by tools/prof_summary.py / pmc_summary.py /
# sq_summary.py. Every step has its own time limit; the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
step() { echo "=== $1 $(date +%T)"; }
step bench_c4; timeout -k 10 300 python bench.py > $O/bench_c4.log 2>&1 || { echo BENCH_C4_FAIL; tail -5 $O/bench_c4.log; exit 1; }
step bench_c1; timeout -k 10 200 python bench.py --config C1 > $O/bench_c1.log 2>&1 || { echo BENCH_C1_FAIL; exit 1; }
step bench_c3; timeout -k 10 200 python bench.py --config C3 > $O/bench_c3.log 2>&1 || { echo BENCH_C3_FAIL; exit 1; }
step bench_c2; timeout -k 10 200 python bench.py --config C2 --no-cpu-baseline > $O/bench_c2.log 2>&1 || { echo BENCH_C2_FAIL; exit 1; }
step bench_c5; timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --steps 10 > $O/bench_c5.log 2>&1 || { echo BENCH_C5_FAIL; exit 1; }
step kt_c4; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 20 --no-profile --no-cpu-baseline > $O/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
step kt_c5; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt5 -o kt5 -- python3 bench.py --config C5 --steps 10 --no-profile --no-cpu-baseline > $O/kt5.log 2>&1 || { echo KT5_FAIL; exit 1; }
step pmc_f; timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o f -- python3 bench.py --steps 10 --warmup 1 --no-profile --no-cpu-baseline > $O/pmc_f.log 2>&1 || { echo PMC_F_FAIL; exit 1; }
step pmc_w; timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o w -- python3 bench.py --steps 10 --warmup 1 --no-profile --no-cpu-baseline > $O/pmc_w.log 2>&1 || { echo PMC_W_FAIL; exit 1; }
step sq; timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH --output-format csv -d $O/sq -o sq -- python3 bench.py --steps 5 --warmup 1 --no-profile --no-cpu-baseline > $O/sq.log 2>&1 || { echo SQ_FAIL; exit 1; }
step stamps_bcr; MIBA_BCR_STAMPS=1 timeout -k 10 120 python tools/kernel_stamps.py C4 3 > $O/stamps_bcr_c4.log 2>&1 || { echo STAMPS_FAIL; exit 1; }
step stamps_tail; MIBA_BCR_STAMPS=1 timeout -k 10 120 python tools/kernel_stamps.py C1 3 > $O/stamps_tail_c1.log 2>&1 || { echo STAMPS_TAIL_FAIL; exit 1; }
echo PROFILE_OK
