#!/bin/bash
# Round 6, lease H: what the z split costs -- the same shapes with the shipped
# library and with the tuning build whose cut lanes skip the hand-over stores
# (GCMX_ZS_NOSEAM: wrong results, timing only), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/h
mkdir -p $OUT
for rep in 1 2; do
  for v in main:gcm_amd/lib/libgcmx.so noseam:gcm_amd/lib/tune/noseam/libgcmx.so; do
    tag=${v%%:*}; lib=${v#*:}
    GCMX_LIB=$lib timeout -k 10 300 python scripts/bench_shape.py 512,512,1024 1024,1024,512 > $OUT/shapes_${tag}_$rep.jsonl 2> $OUT/shapes_${tag}_$rep.err || { echo "$tag rc=$?"; tail -3 $OUT/shapes_${tag}_$rep.err; exit 1; }
    echo "== $tag $rep"; cut -c1-160 $OUT/shapes_${tag}_$rep.jsonl
  done
done
