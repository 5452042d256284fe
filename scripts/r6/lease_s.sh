#!/bin/bash
# Round 6 lease S: two generations of rows at 256^3 (GCMX_TX2_GEN2 = the old
# blocks' share in percent): parity at 256^3 with the split on, then A/B of the
# share, alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/s
mkdir -p $OUT
GCMX_TX2_GEN2=60 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k full_size_256 > $OUT/pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 1 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 0 56 60 64 68; do
    GCMX_TX2_GEN2=$v timeout -k 10 120 python scripts/bench_shape.py 256,256,256 --steps 20 --reps 5 > $OUT/g${v}_$i.json 2> $OUT/g${v}_$i.err || { echo "$v rc=$?"; exit 1; }
    echo "$v $i $(cut -c1-160 $OUT/g${v}_$i.json)"
  done
done
