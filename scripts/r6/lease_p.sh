#!/bin/bash
# Round 6, lease P: face conditions and the folded ODE in the z-split step (rows
# of 1024): parity, then 1024^3 with free surfaces on every face (one pass now;
# before, three per-stage passes) beside the plain step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/p
mkdir -p $OUT
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_faces.py tests/test_gpu_engine.py tests/test_gpu_parity.py tests/test_gpu_slabs.py -k "z1024 or zsplit or ode_fused" > $OUT/pytest_zsf.txt 2>&1
rc=$?; echo "z-split faces rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_zsf.txt | sed 's/ *\[.*//' | tail -20; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 $PT tests/test_gpu_faces.py tests/test_gpu_fma.py tests/test_gpu_layout.py > $OUT/pytest_faces_fma_layout.txt 2>&1
rc=$?; echo "faces+fma+layout rc=$rc"; tail -1 $OUT/pytest_faces_fma_layout.txt; [ $rc -eq 0 ] || { grep -E "^FAILED" $OUT/pytest_faces_fma_layout.txt | head; exit 1; }
timeout -k 10 400 python scripts/bench_shape.py --free 1024,1024,1024 > $OUT/shape_free1024.jsonl 2> $OUT/shape_free1024.err || { echo "free1024 rc=$?"; tail -3 $OUT/shape_free1024.err; exit 1; }
cut -c1-220 $OUT/shape_free1024.jsonl
timeout -k 10 300 python scripts/bench_shape.py 1024,1024,1024 > $OUT/shape_1024.jsonl 2> $OUT/shape_1024.err || exit 1
cut -c1-220 $OUT/shape_1024.jsonl
