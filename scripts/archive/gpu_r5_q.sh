#!/bin/bash
# Round 5, lease Q: the physically contiguous allocation (GCMX_ALLOC=contiguous)
# reproduces the slow 512^3 state on any box; sweep the layout's strides in it
# (row / plane / component padding, tune/cspad build) for a layout that stays
# fast whatever the physical placement; the best ones also with hipMalloc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-q}
mkdir -p $OUT
LIBV=gcm_amd/lib/tune/cspad/libgcmx.so
[ -n "$PADTEST" ] && GCMX_LIB=$LIBV GCMX_ALLOC=contiguous GCMX_ROW_PAD=16 GCMX_PLANE_PAD=64 GCMX_CS_PAD=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fma.py -q --timeout 120 --timeout-method thread > $OUT/pytest_pad.txt 2>&1
rc=$?; echo "pytest (padded layout) rc=$rc"; tail -2 $OUT/pytest_pad.txt
BA="--steps 30 --warmup 5 --reps 3 --no-cpu-baseline --no-copy-ceiling"
b() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py $BA > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,statistics,sys;d=json.load(open(sys.argv[1]));s=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (s.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], 'power', (s.get('power_w') or {}).get('median'), 'sclk', statistics.median(sc) if sc else None, d['process_state']['box'].get('unique_id'))" $OUT/b_$tag.json $tag
}
C="GCMX_LIB=$LIBV GCMX_ALLOC=contiguous"
b main GCMX_NONE=1
b c_base $C
for rp in 16 32 64 128; do b c_row$rp $C GCMX_ROW_PAD=$rp; done
for pp in 16 64 256 1024 4096; do b c_plane$pp $C GCMX_PLANE_PAD=$pp; done
for cp in 64 512 4096; do b c_cs$cp $C GCMX_CS_PAD=$cp; done
b c_base2 $C
