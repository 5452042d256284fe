#!/bin/bash
# One-rank slab timing (scripts/bench_slab.py: the X-slab schedule without
# transfers) over interior rows x boundary rows; output gpurun_out/slab/sweep.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/slab
for br in 8 16 32; do
  for r in 0 24 32; do
    GCMX_BOUNDARY_ROWS=$br timeout -k 10 120 python scripts/bench_slab.py --ranks 8,4 --rows $r --no-check \
      | sed "s/}$/, \"boundary_rows\": $br}/" >> gpurun_out/slab/sweep.jsonl || exit 1
  done
done
timeout -k 10 120 python scripts/bench_slab.py --ranks 8 --sched single --no-check >> gpurun_out/slab/sweep.jsonl || exit 1
cat gpurun_out/slab/sweep.jsonl
