# A/B timing of env-selected variants on C4 (bench breakdown + timed value), no parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/ab_$name.log; return 1; }
  python - "$name" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/ab_{sys.argv[1]}.log').read().strip().splitlines()[-1])
k=d['kernel_ms_per_step']
print(f"{sys.argv[1]:14s} {d['value']:9.1f} it/s {d['ms_per_step']*1e3:7.1f} us/it |", " ".join(f"{n}={v*1e3:.1f}" for n,v in k.items()))
PY
}
