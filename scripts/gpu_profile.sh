#!/bin/bash
# rocprofv3 evidence for the bench configuration: kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md
# §rocprofv3 PMC slots), optional SQ/TCC passes (SQ=1) and, with CALIB=1, the
# same counters on a known-byte calibration stream (tools/calib_fetch) for the
# 8-byte-per-lane access width (otherwise the stored calibration in
# profiles/pmc_traffic.json is reused by tools/pmc_traffic.py).
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
if [ "${SQ:-0}" = 1 ]; then
  i=0
  for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" \
             "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/sq$i -o run -- \
      python3 bench.py --n $N --steps 3 --warmup 1 --no-cpu-baseline --no-profile \
      > $OUT/sq$i.json 2> $OUT/sq$i.err || { echo "sq pass $i failed rc=$?"; exit 1; }
    echo "sq pass $i ok"
  done
fi
if [ "${CALIB:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- \
    ./tools/calib_fetch > $OUT/calib.log 2>&1 || { echo "calib fetch failed rc=$?"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o run -- \
    ./tools/calib_fetch >> $OUT/calib.log 2>&1 || { echo "calib write failed rc=$?"; exit 1; }
  echo "calib ok"
fi
find $OUT -name "*.csv" | head -50
