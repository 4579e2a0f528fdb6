# Same-box A/B of libmiba builds and/or environment settings: bench value + per-kernel ms, alternating the
# variants to cancel clock drift. usage: bash tools/ab_run.sh "label=lib[:ENV=V[:ENV=V]] ..." [rounds] [config]
# (lib = abl/libmiba_<lib>.so; "cur" = the in-tree build)
set -o pipefail
cd $GRAFT_REPO_ROOT
rounds=${2:-3}; cfg=${3:-C4}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for spec in $1; do
    label=${spec%%=*}; rest=${spec#*=}
    IFS=':' read -ra parts <<< "$rest"
    lib=${parts[0]}
    envs=()
    for kv in "${parts[@]:1}"; do envs+=("$kv"); done
    if [ "$lib" = "cur" ]; then libp=$PWD/3dsmc-bundle-adjustment_amd/lib/libmiba.so; else libp=$PWD/abl/libmiba_$lib.so; fi
    env MIBA_LIB_PATH=$libp "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg > gpurun_out/ab_${label}_$r.log 2>&1 || { echo "FAIL $label"; tail -5 gpurun_out/ab_${label}_$r.log; exit 1; }
    python - "$label" "$r" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log').read().strip().splitlines()[-1])
k=d.get('kernel_ms_per_step') or {}
print(f"{sys.argv[1]:10s} {d['value']:9.1f} {d['ms_per_step']*1e3:7.1f} us/it setup={d.get('setup_ms')} dom={d.get('roofline',{}).get('kernel')} {d.get('roofline',{}).get('avg_launch_ms',0)*1e3:.1f} |", " ".join(f"{n}={v*1e3:.1f}" for n,v in k.items()), flush=True)
PY
  done
done
