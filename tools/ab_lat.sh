# Same-box A/B of the TUM-size latency bench (bench.py --config C1 / C3): us per LM iteration of a full solve and of a
# re-solve, alternating the variants. usage: bash tools/ab_lat.sh "label=lib[:ENV=V...] ..." [rounds] [config]
# (lib = abl/libmiba_<lib>.so; "cur" = the in-tree build)
set -o pipefail
cd $GRAFT_REPO_ROOT
rounds=${2:-3}; cfg=${3:-C1}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for spec in $1; do
    label=${spec%%=*}; rest=${spec#*=}
    IFS=':' read -ra parts <<< "$rest"
    lib=${parts[0]}
    envs=()
    for kv in "${parts[@]:1}"; do envs+=("$kv"); done
    if [ "$lib" = "cur" ]; then libp=$PWD/3dsmc-bundle-adjustment_amd/lib/libmiba.so; else libp=$PWD/abl/libmiba_$lib.so; fi
    env MIBA_LIB_PATH=$libp "${envs[@]}" timeout -k 10 200 python bench.py --config $cfg > gpurun_out/abl_${label}_$r.log 2>&1 || { echo "FAIL $label"; tail -5 gpurun_out/abl_${label}_$r.log; exit 1; }
    python - "$label" "$r" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/abl_{sys.argv[1]}_{sys.argv[2]}.log').read().strip().splitlines()[-1])
it=max(d['lm_iterations'],1)
print(f"{sys.argv[1]:8s} solve {d['value']:.4f} ms  {d['value']*1e3/it:6.2f} us/it | resolve {d['ms_per_resolve_prepared']*1e3/it:6.2f} us/it | repeat {d['ms_per_repeat_solve']:.4f} ms |", " ".join(f"{n}={v:.1f}" for n,v in d['kernel_us_per_lm_iteration'].items()), flush=True)
PY
  done
done
