#!/bin/bash
# SQ counter passes (no tracing domains) on the bench kernels, 256^3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq_${TAG:-a}
mkdir -p $OUT
BA="--n ${N:-256} --steps 3 --warmup 1 --no-cpu-baseline --no-profile"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 bench.py $BA \
     > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok"
done
