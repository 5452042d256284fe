#!/bin/bash
# Round 6 lease R: per-block timing of the one-pass step (tune build
# GCMX_TX2_BLKT=1): block durations, end-time spread, per-CU busy time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/r
mkdir -p $OUT
export GCMX_LIB=gcm_amd/lib/tune/blkt/libgcmx.so
timeout -k 10 200 python scripts/r6/diag_blk.py 512 --out $OUT/blk512.npz > $OUT/blk512.jsonl 2> $OUT/blk512.err || { echo rc=$?; tail -n 5 $OUT/blk512.err; exit 1; }
cat $OUT/blk512.jsonl
timeout -k 10 200 python scripts/r6/diag_blk.py 512 --rows 128 --out $OUT/blk512_r128.npz > $OUT/blk512_r128.jsonl 2> $OUT/blk512_r128.err || exit 1
cat $OUT/blk512_r128.jsonl
timeout -k 10 200 python scripts/r6/diag_blk.py 256 --out $OUT/blk256.npz > $OUT/blk256.jsonl 2> $OUT/blk256.err || exit 1
cat $OUT/blk256.jsonl
unset GCMX_LIB
timeout -k 10 200 python scripts/bench_shape.py 512,512,512 --steps 5 --reps 3
