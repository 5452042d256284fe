#!/bin/bash
# Round 5, lease S: chunk size of the shuffled mapping (GCMX_ALLOC=shuffle:<MiB>)
# at 512^3 and 256^3, the N = 8 slab and the 2-D step under it, against hipMalloc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-s}
mkdir -p $OUT
LIBV=gcm_amd/lib/tune/cspad/libgcmx.so
b() {
  tag=$1; n=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --n $n --steps 30 --warmup 5 --reps 3 --no-cpu-baseline --no-copy-ceiling > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,statistics,sys;d=json.load(open(sys.argv[1]));s=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (s.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], 'power', (s.get('power_w') or {}).get('median'), 'sclk', statistics.median(sc) if sc else None, d['process_state']['box'].get('unique_id'))" $OUT/b_$tag.json $tag
  grep -i "failed" $OUT/b_$tag.err | head -2
}
b main512 512 GCMX_NONE=1
for mb in 32 64 128 256 512 1024; do b s${mb}_512 512 GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:$mb; done
b main256 256 GCMX_NONE=1
for mb in 8 16 32 64 128 256; do b s${mb}_256 256 GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:$mb; done
GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:128 timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8_s128.json 2> $OUT/slab8_s128.err || { echo "slab rc=$?"; exit 1; }
tail -1 $OUT/slab8_s128.json | cut -c1-400
timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8_main.json 2> $OUT/slab8_main.err || { echo "slab rc=$?"; exit 1; }
tail -1 $OUT/slab8_main.json | cut -c1-400
GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:128 timeout -k 10 300 python scripts/bench_2d.py --steps 50 > $OUT/b2d_s128.jsonl 2> $OUT/b2d_s128.err || { echo "2d rc=$?"; exit 1; }
grep 8192 $OUT/b2d_s128.jsonl | cut -c1-300
b main512b 512 GCMX_NONE=1
