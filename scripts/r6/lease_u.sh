#!/bin/bash
# Round 6 lease U: wave priority raised while a row's loads issue (tune build
# GCMX_TX2_PRIO=1) against the product build, alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/u
mkdir -p $OUT
for i in 1 2 3; do
  for v in base prio1; do
    if [ $v = base ]; then unset GCMX_LIB; else export GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so; fi
    timeout -k 10 150 python scripts/bench_shape.py 512,512,512 256,256,256 --steps 10 --reps 5 > $OUT/${v}_$i.jsonl 2> $OUT/${v}_$i.err || { echo "$v rc=$?"; tail -n 3 $OUT/${v}_$i.err; exit 1; }
    echo "$v $i"; cut -c1-130 $OUT/${v}_$i.jsonl
  done
done
