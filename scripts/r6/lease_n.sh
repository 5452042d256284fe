#!/bin/bash
# Round 6, lease N: z-split block order -- the parts of a (pair, chunk) adjacent
# (shipped) against pairs fastest (tuning build GCMX_ZS_PAIRS_FIRST=1: an XCD's
# concurrent blocks cover twice as many consecutive x pairs of one part, so
# fewer neighbour planes are fetched twice), 1024^3, rows 128 / 256, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/n
mkdir -p $OUT
GCMX_LIB=gcm_amd/lib/tune/zsp/libgcmx.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slabs.py -k zsplit > $OUT/pytest_zsp.txt 2>&1
rc=$?; echo "zsp parity rc=$rc"; tail -1 $OUT/pytest_zsp.txt; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in main:gcm_amd/lib/libgcmx.so zsp:gcm_amd/lib/tune/zsp/libgcmx.so; do
    tag=${v%%:*}; lib=${v#*:}
    for r in 128 256; do
      GCMX_LIB=$lib timeout -k 10 300 python scripts/bench_shape.py --rows $r 1024,1024,1024 > $OUT/s_${tag}_r${r}_$rep.jsonl 2> $OUT/s_${tag}_r${r}_$rep.err || { echo "$tag rc=$?"; exit 1; }
      echo "$tag r$r rep $rep $(cut -c1-110 $OUT/s_${tag}_r${r}_$rep.jsonl)"
    done
  done
done
