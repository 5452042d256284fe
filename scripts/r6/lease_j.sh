#!/bin/bash
# Round 6, lease J: process-to-process spread of the 256^3 step (fresh process
# each run: a new physical placement) with 16 / 32 / 64 MiB shuffled chunks,
# interleaved; 512^3 with 128 / 256 MiB chunks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/j
mkdir -p $OUT
B="--n 256 --steps 100 --warmup 20 --reps 3 --no-cpu-baseline --no-copy-ceiling --no-box-state --no-clock-probe"
for rep in 1 2 3 4 5; do
  for c in 16 32 64; do
    GCMX_ALLOC=shuffle:$c timeout -k 10 120 python bench.py $B > $OUT/b256_c${c}_$rep.json 2> $OUT/b256_c${c}_$rep.err || { echo "c$c rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b256_c${c}_$rep.json'));r=d['roofline'];print('256 c$c rep $rep',r['kernel_avg_ms'],r['frac'])"
  done
done
B5="--steps 20 --warmup 5 --reps 3 --no-cpu-baseline --no-copy-ceiling --no-box-state --no-clock-probe"
for rep in 1 2 3; do
  for c in 128 256; do
    GCMX_ALLOC=shuffle:$c timeout -k 10 120 python bench.py $B5 > $OUT/b512_c${c}_$rep.json 2> $OUT/b512_c${c}_$rep.err || { echo "c$c rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b512_c${c}_$rep.json'));r=d['roofline'];print('512 c$c rep $rep',r['kernel_avg_ms'],r['frac'])"
  done
done
