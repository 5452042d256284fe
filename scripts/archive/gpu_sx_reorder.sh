#!/bin/bash
# Inner list with the wn-reading nodes last: parity, then the one-launch stage
# against separate launches at 16^3 and (uncapped, mode 3) 64^3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ro && rm -f gpurun_out/ro/b.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_simplex.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ro/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ro/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for f in 1 0; do
  timeout -k 10 200 python scripts/bench_simplex.py --n 16 --steps 400 --warmup 10 --workloads cube,fracture --fusion $f >> gpurun_out/ro/b.jsonl || exit 1
done; done
for f in 3 0; do
  timeout -k 10 200 python scripts/bench_simplex.py --n 64 --steps 30 --warmup 3 --workloads cube,fracture --lanes 8 --fusion $f >> gpurun_out/ro/b.jsonl || exit 1
done
timeout -k 10 200 python scripts/bench_simplex.py --n 64 --steps 30 --warmup 3 --workloads cube,fracture --lanes 1 >> gpurun_out/ro/b.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/ro/b.jsonl'):
    r = json.loads(l); print(r['mesh'][:22], r['workload'], 'lanes', r['lanes'], 'fusion', r['fusion'], r['fused_stages'], r['ms_per_step'])"
