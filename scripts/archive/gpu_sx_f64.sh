#!/bin/bash
# Simplex layouts at 32^3-64^3: eight lanes with the one-launch stage (automatic
# below 131 072 vertices, grid cap 4 096 blocks) against one thread per node.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/f64 && rm -f gpurun_out/f64/b.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_simplex.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f64/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/f64/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 32 48; do
  for l in 0 1; do
    timeout -k 10 200 python scripts/bench_simplex.py --n $n --steps 60 --warmup 3 --workloads cube,fracture,layered --lanes $l >> gpurun_out/f64/b.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('gpurun_out/f64/b.jsonl'):
    r = json.loads(l); print(r['mesh'][:30], r['workload'], r['vertices'], 'lanes', r['lanes'], 'fusion', r['fusion'], r['fused_stages'], r['ms_per_step'], r['value'])"
