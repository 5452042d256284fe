#!/bin/bash
# Round 5, lease H (diagnostics): SQ counter passes of the current 512^3 step
# (rocprofv3 --pmc, one pass per set) and the per-wave phase cycles of the
# exact build's k_step_tx2 (tuning build with GCMX_TX2_DIAG=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-h}
mkdir -p $OUT
GCMX_FP=exact GCMX_LIB=gcm_amd/lib/tune/diag/libgcmx.so timeout -k 10 200 python scripts/tx2_diag.py > $OUT/diag_exact.txt 2>&1; echo "diag rc=$?"; cat $OUT/diag_exact.txt
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/sq$i -o run -- \
    python3 bench.py --n 512 --steps 3 --warmup 1 --reps 3 --no-cpu-baseline --no-profile --no-copy-ceiling --no-box-state \
    > $OUT/sq$i.json 2> $OUT/sq$i.err || { echo "sq pass $i failed rc=$?"; exit 1; }
  echo "sq pass $i ok"
done
