#!/bin/bash
# Round-3 GPU check: the whole -m gpu suite in one process, smoke, the default
# bench line, and the X-slab group emulation at K = 2, 4, 8 (bench.py
# --emulate-slabs).  Output under gpurun_out/r3/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/${TAG:-run}
mkdir -p $OUT
set -o pipefail
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 1100 python -u -m pytest tests/ -m gpu -x -v --timeout 900 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python bench.py > $OUT/bench_512.json 2> $OUT/bench_512.err || { echo "bench rc=$?"; tail $OUT/bench_512.err; exit 1; }
cat $OUT/bench_512.json
timeout -k 10 200 python bench.py --n 256 --steps 50 --no-cpu-baseline > $OUT/bench_256.json 2> $OUT/bench_256.err || { echo "bench256 rc=$?"; exit 1; }
cat $OUT/bench_256.json
for K in ${SLABS:-8 4 2}; do
  timeout -k 10 300 python bench.py --emulate-slabs $K --steps 10 --reps 5 > $OUT/emulate_$K.json 2> $OUT/emulate_$K.err || { echo "emulate $K rc=$?"; tail $OUT/emulate_$K.err; exit 1; }
  cat $OUT/emulate_$K.json
done
