#!/bin/bash
# Round 6 lease V: rows per k_zseam block (GCMX_ZSEAM_ROWS 64 / 32 / 16) at
# 1024^3, parity of the z split under each, and the two-generation face case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_faces.py -k "gen2 or z1024" > $OUT/pytest_faces.txt 2>&1; rc=$?; echo "faces rc=$rc"; tail -n 1 $OUT/pytest_faces.txt
[ $rc -eq 0 ] || exit $rc
for v in 32 16; do
  GCMX_ZSEAM_ROWS=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_faces.py -k "zsplit or z1024" > $OUT/pytest_zs$v.txt 2>&1; rc=$?; echo "zs$v rc=$rc"; tail -n 1 $OUT/pytest_zs$v.txt
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for v in 64 32 16; do
    GCMX_ZSEAM_ROWS=$v timeout -k 10 200 python scripts/bench_shape.py 1024,1024,1024 --steps 5 --reps 3 > $OUT/z${v}_$i.json 2> $OUT/z${v}_$i.err || { echo "$v rc=$?"; exit 1; }
    echo "$v $i $(cut -c1-150 $OUT/z${v}_$i.json)"
  done
done
