#!/bin/bash
# Round 6 lease W: SIMD partners holding neighbouring z blocks (tune build
# GCMX_TX2_ZPERM=1): parity with that library, then 512^3 A/B alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/w
mkdir -p $OUT
[ -n "$SKIP_PARITY" ] || GCMX_LIB=gcm_amd/lib/tune/zperm/libgcmx.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fma.py tests/test_gpu_faces.py > $OUT/pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 1 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4 5 6; do
  for v in base zperm; do
    if [ $v = base ]; then unset GCMX_LIB; else export GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so; fi
    timeout -k 10 150 python scripts/bench_shape.py 512,512,512 --steps 10 --reps 5 > $OUT/${v}_$i.jsonl 2> $OUT/${v}_$i.err || { echo "$v rc=$?"; tail -n 3 $OUT/${v}_$i.err; exit 1; }
    echo "$v $i $(cut -c1-130 $OUT/${v}_$i.jsonl)"
  done
done
