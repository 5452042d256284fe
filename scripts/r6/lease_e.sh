#!/bin/bash
# Round 6, lease E: rows per block and chunk size of the 1024^3 z-split step;
# the 256^3 rows-per-block rule under the shuffled placement (alternating
# repetitions); one N = 8 slab rank with the exchange through the loopback
# transport at 40 / 50 / 56 / 64 GB/s per direction (where the exchange stops
# hiding behind the interior).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/e
mkdir -p $OUT
B1="--n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling"
for v in "r128::--rows-per-block 128" "r256::--rows-per-block 256" "r256g1:GCMX_ALLOC=shuffle:1024:--rows-per-block 256" "r256m:GCMX_ALLOC=malloc:--rows-per-block 256" "r256g512:GCMX_ALLOC=shuffle:512:--rows-per-block 256" "r64::--rows-per-block 64"; do
  tag=${v%%:*}; rest=${v#*:}; envs=${rest%%:--*}; arg=--${rest#*:--}
  [ "$envs" = "$rest" ] && envs=""
  env $envs timeout -k 10 400 python bench.py $B1 $arg > $OUT/b1024_$tag.json 2> $OUT/b1024_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b1024_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b1024_$tag.json'));r=d['roofline'];print('1024 $tag',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],d['process_state']['layers']['alloc'])"
done
B2="--n 256 --steps 100 --warmup 20 --reps 5 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2; do for r in 32 64 128; do
  timeout -k 10 200 python bench.py $B2 --rows-per-block $r > $OUT/b256_r${r}_$rep.json 2> $OUT/b256_r${r}_$rep.err || { echo "bench 256 r$r rc=$?"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b256_r${r}_$rep.json'));r=d['roofline'];print('256 rows $r rep $rep',d['ms_per_step'],r['kernel_avg_ms'],r['frac'])"
done; done
for g in 40 50 56 64; do
  timeout -k 10 300 python scripts/bench_slab.py --ranks 8 --loop-gbps $g --no-check > $OUT/slab8_loop$g.json 2> $OUT/slab8_loop$g.err || { echo "slab loop $g rc=$?"; tail -3 $OUT/slab8_loop$g.err; exit 1; }
  tail -1 $OUT/slab8_loop$g.json | cut -c1-600
done
