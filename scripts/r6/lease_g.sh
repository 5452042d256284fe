#!/bin/bash
# Round 6, lease G: the z split with the cut lanes' stores moved behind the row's
# stores; shapes separating the z split's cost from the grid size
# (1024 x 1024 x 512 runs the unsplit step on the same node count as half of 1024^3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/g
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slabs.py -k "zsplit" > $OUT/pytest_zs.txt 2>&1
rc=$?; echo "zsplit parity rc=$rc"; tail -1 $OUT/pytest_zs.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/bench_shape.py 512,512,512 1024,1024,512 512,512,1024 1024,1024,1024 > $OUT/shapes.jsonl 2> $OUT/shapes.err || { echo "shapes rc=$?"; tail -3 $OUT/shapes.err; exit 1; }
cat $OUT/shapes.jsonl
GCMX_ZS_PART=256 timeout -k 10 300 python scripts/bench_shape.py 512,512,512 512,512,1024 > $OUT/shapes_zs256.jsonl 2> $OUT/shapes_zs256.err || { echo "shapes zs256 rc=$?"; exit 1; }
cat $OUT/shapes_zs256.jsonl
GCMX_ZS_PART=256 timeout -k 10 300 python scripts/bench_shape.py --rows 512 512,512,512 > $OUT/shapes_zs256_r512.jsonl 2> $OUT/shapes_zs256_r512.err || { echo "shapes zs256 r512 rc=$?"; exit 1; }
cat $OUT/shapes_zs256_r512.jsonl
