#!/bin/bash
# Round 4, lease i: the HET ODE fold (parity + 256^3 rate) and the suites it touches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/${LEASE:-i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slabs.py \
  tests/test_gpu_engine.py tests/test_gpu_fma.py tests/test_gpu_faces.py -m gpu > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -30; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for a in "hetmax:--layers --maxwell" "max:--maxwell" "het:--layers"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 200 python3 scripts/bench_physics.py --n 256 --steps 30 $args > $OUT/phys_$n.json 2> $OUT/phys_$n.err || { echo "$n rc=$?"; exit 1; }
  tail -1 $OUT/phys_$n.json
done
