#!/bin/bash
# Round 5, lease AA: process-to-process spread of the shuffled placement at
# 512^3: 64 MiB against 256 MiB chunks, six fresh processes each, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-aa}
mkdir -p $OUT
for rep in 1 2 3 4 5 6; do
  for mb in 64 256; do
    GCMX_ALLOC=shuffle:$mb timeout -k 10 300 python bench.py --steps 20 --warmup 3 --reps 5 --no-cpu-baseline --no-copy-ceiling --no-box-state --no-clock-probe > $OUT/b_${mb}_$rep.json 2> $OUT/b_${mb}_$rep.err || { echo "rc=$?"; exit 1; }
    python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $OUT/b_${mb}_$rep.json "s$mb r$rep"
  done
done
