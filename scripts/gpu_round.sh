#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Stops at the first GPU
# fault / abort / timeout; plain test failures (exit 1) still let the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok_or_stop() {  # $1 = rc, $2 = step name
  case "$1" in
    0|1) return 0 ;;
    *) echo "STOP after $2 (rc=$1)"; exit "$1" ;;
  esac
}
timeout -k 10 900 python -m pytest tests -q -m gpu -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok_or_stop $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok_or_stop $rc smoke
for n in ${BENCH_SIZES:-256 512}; do
  timeout -k 10 400 python bench.py --n $n ${BENCH_ARGS} > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err
  rc=$?; echo "bench n=$n rc=$rc"; cat gpurun_out/bench_$n.json; tail -3 gpurun_out/bench_$n.err
  [ $rc -eq 0 ] || exit $rc
done
