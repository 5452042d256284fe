#!/bin/bash
# Round-3 schedule / block-shape sweep on one MI355X: slab parity of the
# boundary-first schedule, per-rank slab times (bench_slab.py) for the X-slab
# and boundary-first schedules, and rows-per-block A/B of the 512^3 / 256^3
# step.  Output under gpurun_out/r3/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/${TAG:-sched}
mkdir -p $OUT
set -o pipefail
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_slabs.py tests/test_gpu_parity.py -m gpu -x -v \
    -k "slab and not eight" --timeout 500 --timeout-method thread > $OUT/pytest_slabs.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_slabs.log
  [ $rc -eq 0 ] || exit $rc
fi
for BR in ${BROWS:-4 8}; do
  for R in ${ROWS:-0 32 64}; do
    GCMX_BOUNDARY_ROWS=$BR timeout -k 10 200 python scripts/bench_slab.py --sched bfirst --rows $R --ranks 8,4 --no-check \
      >> $OUT/slab_bfirst.jsonl 2>> $OUT/slab.err || { echo "bench_slab rc=$?"; tail $OUT/slab.err; exit 1; }
  done
done
timeout -k 10 200 python scripts/bench_slab.py --sched xslab --ranks 8,4 --no-check >> $OUT/slab_xslab.jsonl 2>> $OUT/slab.err || exit 1
timeout -k 10 200 python scripts/bench_slab.py --sched single --ranks 8,4 --no-check >> $OUT/slab_single.jsonl 2>> $OUT/slab.err || exit 1
cat $OUT/slab_bfirst.jsonl $OUT/slab_xslab.jsonl $OUT/slab_single.jsonl
for R in ${ROWS512:-0 512 0 512}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-copy-ceiling --rows-per-block $R --reps 5 \
    >> $OUT/bench_512_rows.jsonl 2>> $OUT/bench.err || { echo "bench rc=$?"; tail $OUT/bench.err; exit 1; }
done
for R in ${ROWS256:-0 32 128 0}; do
  timeout -k 10 200 python bench.py --n 256 --steps 50 --no-cpu-baseline --no-copy-ceiling --rows-per-block $R --reps 5 \
    >> $OUT/bench_256_rows.jsonl 2>> $OUT/bench.err || { echo "bench256 rc=$?"; tail $OUT/bench.err; exit 1; }
done
python - <<'EOF' $OUT
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*_rows.jsonl")):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1], d["config"].get("rows_per_block"), d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel_avg_ms"])
EOF
