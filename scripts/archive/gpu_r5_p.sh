#!/bin/bash
# Round 5, lease P: the 512^3 step against the component-plane stride (cs
# padded by GCMX_CS_PAD elements) and the allocation (hipMalloc or physically
# contiguous), tune/cspad build; main build first and last.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-p}
mkdir -p $OUT
BA="--steps 30 --warmup 5 --reps 3 --no-cpu-baseline --no-copy-ceiling"
b() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py $BA > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,statistics,sys;d=json.load(open(sys.argv[1]));s=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (s.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], 'power', (s.get('power_w') or {}).get('median'), 'sclk', statistics.median(sc) if sc else None, d['process_state']['box'].get('unique_id'))" $OUT/b_$tag.json $tag
}
L=GCMX_LIB=gcm_amd/lib/tune/cspad/libgcmx.so
b main0 GCMX_NONE=1
for pad in 0 512 8192 131072 262144 1048576 3000064; do
  b pad$pad $L GCMX_CS_PAD=$pad
done
b contig0 $L GCMX_ALLOC=contiguous
b contig131072 $L GCMX_ALLOC=contiguous GCMX_CS_PAD=131072
b main1 GCMX_NONE=1
