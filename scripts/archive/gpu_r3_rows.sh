#!/bin/bash
# Rows per block of the one-pass step (FMA build) at 256^3 and 512^3, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/rows; mkdir -p $OUT
for n in 256 512; do
  for r in 0 32 64 128 256 512; do
    [ $n = 256 ] && [ $r -gt 256 ] && continue
    timeout -k 10 200 python bench.py --n $n --steps 20 --no-cpu-baseline --no-copy-ceiling --rows-per-block $r > $OUT/b_${n}_$r.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $OUT/b_${n}_$r.json $n $r
  done
done
