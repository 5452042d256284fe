#!/bin/bash
# Round 5, lease CC: 1024^3 (k_fused_xyz<2, 1024>) rows per block: 128 (the
# automatic choice), 64, 256, 512.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-cc}
mkdir -p $OUT
for r in 0 64 256 512 0; do
  timeout -k 10 400 python bench.py --n 1024 --steps 5 --warmup 2 --reps 3 --rows-per-block $r --no-cpu-baseline --no-copy-ceiling --no-box-state > $OUT/b1024_r$r.json 2> $OUT/b1024_r$r.err || { echo "r$r rc=$?"; tail -3 $OUT/b1024_r$r.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('rows', sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])" $OUT/b1024_r$r.json $r
done
