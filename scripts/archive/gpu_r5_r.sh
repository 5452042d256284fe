#!/bin/bash
# Round 5, lease R: the layers' block mapped from physical chunks in shuffled
# order (GCMX_ALLOC=shuffle:<MiB>, tune/cspad build) against hipMalloc and the
# physically contiguous allocation (the slow state), 512^3; parity suite under
# the shuffled mapping.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-r}
mkdir -p $OUT
LIBV=gcm_amd/lib/tune/cspad/libgcmx.so
GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_shuffle.txt 2>&1
rc=$?; echo "pytest (shuffle:2) rc=$rc"; tail -2 $OUT/pytest_shuffle.txt; [ $rc -eq 0 ] || exit $rc
BA="--steps 30 --warmup 5 --reps 3 --no-cpu-baseline --no-copy-ceiling"
b() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py $BA > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,statistics,sys;d=json.load(open(sys.argv[1]));s=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (s.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], 'power', (s.get('power_w') or {}).get('median'), 'sclk', statistics.median(sc) if sc else None, d['process_state']['box'].get('unique_id'))" $OUT/b_$tag.json $tag
  grep -i "failed" $OUT/b_$tag.err | head -2
}
b main GCMX_NONE=1
b contig GCMX_LIB=$LIBV GCMX_ALLOC=contiguous
for mb in 2 16 64 256; do b shuffle$mb GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:$mb; done
b contig2 GCMX_LIB=$LIBV GCMX_ALLOC=contiguous
b shuffle2b GCMX_LIB=$LIBV GCMX_ALLOC=shuffle:2
b main2 GCMX_NONE=1
