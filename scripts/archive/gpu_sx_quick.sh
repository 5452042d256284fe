#!/bin/bash
# Simplex iteration on one GPU box: GPU parity tests, per-kernel times of the
# 16^3 cube for the current build and every tuning variant under
# gcm_amd/lib/sxtune (gpu_sx_variants.sh), then the 16^3 cube step with and
# without graph replay.  Output under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_simplex.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sx_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sx_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_sx_variants.sh || exit $?
rm -f gpurun_out/sx16.jsonl
for g in "" "--graph"; do
  timeout -k 10 200 python scripts/bench_simplex.py --n 16 --steps 200 --warmup 5 --workloads cube $g >> gpurun_out/sx16.jsonl || exit $?
done
python3 - <<'PY'
import json
for l in open("gpurun_out/sx16.jsonl"):
    r = json.loads(l)
    print(r["workload"], "graph" if r["graph"] else "calls", r["ms_per_step"], "ms/step")
PY
