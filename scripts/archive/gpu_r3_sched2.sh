#!/bin/bash
# Round-3 schedule check 2: parity of the one-launch boundary sides and the
# rows-per-block rule, per-rank slab times of the three schedules (median of 5
# repetitions), a kernel trace of the boundary-first slab step (idle gaps), and
# the 512^3 / 256^3 bench lines with the new automatic rows per block.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/${TAG:-sched2}
mkdir -p $OUT
set -o pipefail
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_slabs.py tests/test_gpu_parity.py tests/test_gpu_faces.py -m gpu -x -v \
    -k "not eight" --timeout 500 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for S in bfirst xslab single; do
  timeout -k 10 200 python scripts/bench_slab.py --sched $S --ranks 8,4,2 --no-check --steps 30 \
    >> $OUT/slab.jsonl 2>> $OUT/slab.err || { echo "bench_slab rc=$?"; tail $OUT/slab.err; exit 1; }
done
for BR in 2 8; do
  GCMX_BOUNDARY_ROWS=$BR timeout -k 10 200 python scripts/bench_slab.py --sched bfirst --ranks 8 --no-check --steps 30 \
    >> $OUT/slab.jsonl 2>> $OUT/slab.err || { echo "bench_slab rc=$?"; exit 1; }
done
cat $OUT/slab.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o slab8 -- \
  python scripts/bench_slab.py --sched bfirst --ranks 8 --no-check --steps 30 --reps 2 > $OUT/trace.out 2>&1 \
  || { echo "rocprof rc=$?"; tail $OUT/trace.out; exit 1; }
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1); python scripts/trace_gaps.py $f 200 | tee $OUT/trace_gaps.txt
timeout -k 10 300 python bench.py --no-copy-ceiling --cpu-seconds 2 > $OUT/bench_512.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail $OUT/bench.err; exit 1; }
timeout -k 10 200 python bench.py --n 256 --steps 50 --no-cpu-baseline > $OUT/bench_256.json 2>> $OUT/bench.err || { echo "bench256 rc=$?"; exit 1; }
python - <<'EOF' $OUT
import json, sys
for f in ("bench_512.json", "bench_256.json"):
    d = json.load(open(sys.argv[1] + "/" + f))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["frac"], r["kernel_avg_ms"], r["kernel_symbol"], r.get("copy_ceiling", {}).get("frac_of_copy"))
EOF
