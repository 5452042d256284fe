#!/bin/bash
# rocprofv3 evidence for the bench configuration: kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md
# §rocprofv3 PMC slots), then the same counters on a known-byte calibration
# stream (tools/calib_fetch) for the 8-byte-per-lane access width.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r1}
mkdir -p $OUT
N=${N:-512}
BA="--n $N --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline"
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $BA > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed rc=$?"; exit 1; }
echo "trace ok"; cat $OUT/trace_bench.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py $BA --no-profile > $OUT/fetch_bench.json 2> $OUT/fetch.err || { echo "fetch failed rc=$?"; exit 1; }
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py $BA --no-profile > $OUT/write_bench.json 2> $OUT/write.err || { echo "write failed rc=$?"; exit 1; }
echo "write ok"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- \
  ./tools/calib_fetch > $OUT/calib.log 2>&1 || { echo "calib fetch failed rc=$?"; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o run -- \
  ./tools/calib_fetch >> $OUT/calib.log 2>&1 || { echo "calib write failed rc=$?"; exit 1; }
echo "calib ok"
find $OUT -name "*.csv" | head -50
