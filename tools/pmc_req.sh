# TCC read-request size passes for the C4 bench (run on the GPU box from the repo root): lists the
# gfx950 counters, then one --pmc pass per group of TCC request counters that exist on this build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcreq
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || { echo LIST_FAIL; exit 1; }
has() { grep -q -w "$1" $O/avail.txt; }
run() {  # name counters...
    local n=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o $n -- python3 bench.py --steps 10 --warmup 1 --no-profile --no-cpu-baseline > $O/$n.log 2>&1 || { echo PMC_${n}_FAIL; exit 1; }
    echo "pass $n: $*"
}
G1=(); for c in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum; do has ${c%_sum} && G1+=($c); done
G2=(); for c in TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum; do has ${c%_sum} && G2+=($c); done
G3=(); for c in TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum; do has ${c%_sum} && G3+=($c); done
G4=(); for c in TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum; do has ${c%_sum} && G4+=($c); done
[ ${#G1[@]} -gt 0 ] && run rq1 "${G1[@]}"
[ ${#G2[@]} -gt 0 ] && run rq2 "${G2[@]}"
[ ${#G3[@]} -gt 0 ] && run rq3 "${G3[@]}"
[ ${#G4[@]} -gt 0 ] && run rq4 "${G4[@]}"
echo PMCREQ_OK
