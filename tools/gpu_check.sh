# GPU check: parity tests (-m gpu), C4 bench line, BCR timeline stamps. Run from the repo root.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench_c4.log; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/bench_c4.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step']); print(d['kernel_ms_per_step'])
PY
MIBA_BCR_STAMPS=1 timeout -k 10 120 python tools/kernel_stamps.py C4 1 > gpurun_out/stamps_c4.log 2>&1 || echo STAMPS_FAIL
bash tools/ab_run.sh
