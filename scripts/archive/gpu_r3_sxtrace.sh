#!/bin/bash
# Kernel trace of the simplex config-4 task (cube.off, h 0.05) and the 16^3
# cube: per-kernel durations and the idle gaps between launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-sxtrace}
mkdir -p $OUT
set -o pipefail
for W in cubetask cube; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$W -o run -- \
    python3 scripts/bench_simplex.py --workloads $W --n 16 --steps 100 > $OUT/$W.json 2> $OUT/$W.err \
    || { echo "$W rc=$?"; tail $OUT/$W.err; exit 1; }
  f=$(find $OUT/$W -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_gaps.py $f 200 | tee $OUT/${W}_gaps.txt
  cat $OUT/$W.json
done
