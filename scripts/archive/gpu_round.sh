#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.  Stops
# at the first GPU fault / abort / timeout; plain test failures (exit 1) still
# let the bench run.  TAG names the output directory (gpurun_out/$TAG).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
ok_or_stop() {  # $1 = rc, $2 = step name
  case "$1" in
    0|1) return 0 ;;
    *) echo "STOP after $2 (rc=$1)"; exit "$1" ;;
  esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1500 python -u -m pytest tests -v -m gpu -rf --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; ok_or_stop $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; ok_or_stop $rc smoke
fi
for n in ${BENCH_SIZES:-512 256}; do
  timeout -k 10 400 python bench.py --n $n ${BENCH_ARGS} > $OUT/bench_$n.json 2> $OUT/bench_$n.err
  rc=$?; echo "bench n=$n rc=$rc"; cat $OUT/bench_$n.json; tail -3 $OUT/bench_$n.err
  [ $rc -eq 0 ] || exit $rc
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --n 512 --steps 10 --reps 1 --warmup 2 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err
  rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find $OUT/trace -name "*stats*"
fi
