#!/bin/bash
# PMC passes for the fused step kernel, one rocprofv3 run per counter group
# (MI355X_MICROARCH.md: <= 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 GRBM per pass).  LIBS =
# space-separated NAME=path/to/libgcmx.so (default: the in-tree build).  Output:
# gpurun_out/ctr_$TAG/<name>/p<k>/..., summarised by scripts/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr_${TAG:-r2}
mkdir -p $OUT
N=${N:-512}
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum"
  "TCC_BUSY_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS"
)
for spec in ${LIBS:-base=gcm_amd/lib/libgcmx.so}; do
  name="${spec%%=*}"; lib="${spec#*=}"
  k=0
  for set in "${PASSES[@]}"; do
    k=$((k+1)); mkdir -p $OUT/$name
    GCMX_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/$name/p$k -o run -- \
      python3 bench.py --n $N --steps 3 --reps 1 --warmup 1 --no-cpu-baseline --no-profile \
      > $OUT/$name/p$k.json 2> $OUT/$name/p$k.err || { echo "$name pass $k failed rc=$?"; tail -3 $OUT/$name/p$k.err; exit 1; }
    echo "$name pass $k ok"
  done
done
python3 scripts/pmc_summary.py $OUT
