#!/bin/bash
# One-launch simplex stage: GPU parity tests, then the 16^3 cube step with and
# without the fusion (alternating, same box), 64^3 workloads, and a kernel trace
# of the fused 16^3 run.  Output under gpurun_out/sxf/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sxf
timeout -k 10 300 python -u -m pytest tests/test_gpu_simplex.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sxf/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sxf/pytest.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/sxf/b16.jsonl gpurun_out/sxf/b64.jsonl
for r in 1 2; do
  for f in "--fusion 1" "--fusion 2" "--fusion 0"; do
    timeout -k 10 200 python scripts/bench_simplex.py --n 16 --steps 400 --warmup 10 --workloads cube,fracture $f >> gpurun_out/sxf/b16.jsonl || exit $?
  done
done
for f in "--fusion 1" "--fusion 2" "--fusion 0"; do
  timeout -k 10 300 python scripts/bench_simplex.py --n 64 --steps 20 --warmup 2 --workloads cube,fracture --lanes 8 $f >> gpurun_out/sxf/b64.jsonl || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sxf/prof -o run -- python3 scripts/bench_simplex.py --n 16 --steps 200 --warmup 5 --workloads cube > gpurun_out/sxf/prof.log 2>&1 || exit $?
python3 - <<'PY'
import json
for f in ("b16", "b64"):
    for l in open(f"gpurun_out/sxf/{f}.jsonl"):
        r = json.loads(l)
        print(f, r["workload"], "fusion", r["fusion"], r["fused_stages"], r["ms_per_step"], "ms/step", r["value"])
PY
