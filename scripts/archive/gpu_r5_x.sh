#!/bin/bash
# Round 5, lease X: stride padding under the shuffled placement (tune/pad build:
# GCMX_ROW_PAD / GCMX_PLANE_PAD / GCMX_CS_PAD elements), 512^3 and 256^3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-x}
mkdir -p $OUT
b() {
  tag=$1; args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-copy-ceiling > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['process_state']['box'].get('unique_id'))" $OUT/b_$tag.json $tag
}
L=GCMX_LIB=gcm_amd/lib/tune/pad/libgcmx.so
A="--steps 30 --warmup 5 --reps 5"
b main "$A" GCMX_NONE=1
for v in GCMX_ROW_PAD=16 GCMX_ROW_PAD=32 GCMX_PLANE_PAD=16 GCMX_PLANE_PAD=64 GCMX_PLANE_PAD=256 GCMX_PLANE_PAD=4096 GCMX_CS_PAD=512 GCMX_CS_PAD=65536; do
  b ${v/=/_} "$A" $L $v
done
b main2 "$A" GCMX_NONE=1
A="--n 256 --steps 100 --warmup 20 --reps 5"
b main256 "$A" GCMX_NONE=1
for v in GCMX_ROW_PAD=16 GCMX_PLANE_PAD=64 GCMX_PLANE_PAD=4096 GCMX_CS_PAD=512; do
  b ${v/=/_}_256 "$A" $L $v
done
b main256b "$A" GCMX_NONE=1
