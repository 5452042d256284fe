#!/bin/bash
# Simplex: GPU tests (incl. gsx_step graph replay == individual calls) and step
# latency with and without graph replay at the reference's mesh sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/simplex_${TAG:-r2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_simplex.py -v -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -6 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 16 64; do
  for g in "" "--graph"; do
    timeout -k 10 300 python scripts/bench_simplex.py --n $n --steps 50 --warmup 3 $g >> $OUT/bench.jsonl 2>> $OUT/bench.err || exit 1
  done
done
cat $OUT/bench.jsonl
