#!/bin/bash
# Simplex: GPU tests (incl. gsx_step graph replay == individual calls) and step
# latency with and without graph replay at the reference's mesh sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/simplex_${TAG:-r2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_simplex.py -v -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -6 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in ${SIZES:-16 64}; do
  for g in "" "--graph"; do
    for l in 1 8; do
      timeout -k 10 300 python scripts/bench_simplex.py --n $n --steps 50 --warmup 3 --lanes $l $g >> $OUT/bench.jsonl 2>> $OUT/bench.err || exit 1
    done
  done
done
cat $OUT/bench.jsonl
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace16 -o run -- \
    python3 scripts/bench_simplex.py --n 16 --steps 20 --warmup 3 --workloads cube --lanes 8 > $OUT/trace16.json 2> $OUT/trace16.err || exit 1
  python3 - $OUT/trace16/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1000:8.2f} us")
PY
fi
