# Same-box A/B of two libmiba builds (abl/libmiba_<name>.so) on C4: bench value + per-kernel ms,
# alternating builds to cancel clock drift. usage: bash tools/ab_lib.sh "old new ..." [rounds] [config]
set -o pipefail
cd $GRAFT_REPO_ROOT
rounds=${2:-3}; cfg=${3:-C4}
for r in $(seq 1 $rounds); do
  for name in $1; do
    MIBA_LIB_PATH=$PWD/abl/libmiba_$name.so timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/ab_${name}_$r.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/ab_${name}_$r.log; exit 1; }
    python - "$name" "$r" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log').read().strip().splitlines()[-1])
k=d.get('kernel_ms_per_step') or {}
print(f"{sys.argv[1]:8s} {d['value']:9.1f} {d['ms_per_step']*1e3:7.1f} us/it bcr_avg={d.get('roofline',{}).get('avg_launch_ms',0)*1e3:.1f} |", " ".join(f"{n}={v*1e3:.1f}" for n,v in k.items()))
PY
  done
done
