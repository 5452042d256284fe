#!/bin/bash
# Round 6, lease K: shuffled-chunk size for blocks under 8 GiB, fresh process per
# run, interleaved: the N = 8 slab (64 x 512^2, the config-3 rank), 256^3 and the
# 2-D 8192^2 step with 32 against 64 MiB chunks (16 for 256^3 too).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/k
mkdir -p $OUT
for rep in 1 2 3 4; do
  for c in 32 64; do
    GCMX_ALLOC=shuffle:$c timeout -k 10 120 python scripts/bench_slab.py --ranks 8 --no-check --steps 30 > $OUT/slab8_c${c}_$rep.json 2> $OUT/slab8_c${c}_$rep.err || { echo "slab c$c rc=$?"; exit 1; }
    echo "slab8 c$c rep $rep $(tail -1 $OUT/slab8_c${c}_$rep.json | cut -c1-120)"
  done
done
B="--n 256 --steps 100 --warmup 20 --reps 3 --no-cpu-baseline --no-copy-ceiling --no-box-state --no-clock-probe"
for rep in 1 2 3 4; do
  for c in 16 32 64; do
    GCMX_ALLOC=shuffle:$c timeout -k 10 120 python bench.py $B > $OUT/b256_c${c}_$rep.json 2> $OUT/b256_c${c}_$rep.err || { echo "c$c rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b256_c${c}_$rep.json'));r=d['roofline'];print('256 c$c rep $rep',r['kernel_avg_ms'],r['frac'])"
  done
done
for rep in 1 2 3; do
  for c in 32 64; do
    GCMX_ALLOC=shuffle:$c timeout -k 10 200 python scripts/bench_2d.py --steps 50 > $OUT/b2d_c${c}_$rep.jsonl 2> $OUT/b2d_c${c}_$rep.err || { echo "2d c$c rc=$?"; exit 1; }
    echo "2d c$c rep $rep $(sed -n 3p $OUT/b2d_c${c}_$rep.jsonl | cut -c1-160)"
  done
done
