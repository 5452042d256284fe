#!/bin/bash
# Round 5, lease T: the shuffled chunk mapping as the default allocation: full
# GPU suite, then A/B against GCMX_ALLOC=malloc (512^3 x2, 256^3 steady x2),
# alternating, and the N = 8 slab, 2-D and 1024^3 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-t}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -20; exit $rc; }
b() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py $BA > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,statistics,sys;d=json.load(open(sys.argv[1]));s=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (s.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], 'power', (s.get('power_w') or {}).get('median'), 'sclk', statistics.median(sc) if sc else None, d['process_state']['box'].get('unique_id'), d['process_state']['layers']['alloc'])" $OUT/b_$tag.json $tag
}
BA="--steps 30 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2; do b def512_$rep GCMX_NONE=1; b malloc512_$rep GCMX_ALLOC=malloc; done
BA="--n 256 --steps 100 --warmup 20 --reps 7 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2; do b def256_$rep GCMX_NONE=1; b malloc256_$rep GCMX_ALLOC=malloc; done
timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8.json 2> $OUT/slab8.err || { echo "slab rc=$?"; exit 1; }
tail -1 $OUT/slab8.json | cut -c1-330
timeout -k 10 300 python scripts/bench_2d.py --steps 50 > $OUT/b2d.jsonl 2> $OUT/b2d.err || { echo "2d rc=$?"; exit 1; }
grep 8192 $OUT/b2d.jsonl | cut -c1-260
BA="--n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling"
b def1024 GCMX_NONE=1
