#!/bin/bash
# Channels per peer (GCMX_COMM_CHANNELS_PER_PEER) against the slab thickness,
# one-rank RCCL self-exchange, one process per setting.  gpurun_out/r3/rcclch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/rcclch
mkdir -p $OUT
set -o pipefail
# ch = auto: the library's own choice (step_free_cus), one process per slab size
for ch in ${CHS:-3 4 6}; do
  if [ "$ch" = auto ]; then
    : > $OUT/c$ch.jsonl
    for r in ${RANKS:-8 4 2}; do
      timeout -k 10 150 python3 scripts/bench_slab.py --ranks $r --steps 30 --rccl-self --no-check \
        >> $OUT/c$ch.jsonl 2> $OUT/c$ch.err || { tail -5 $OUT/c$ch.err; exit 1; }
    done
  else
  GCMX_COMM_CHANNELS_PER_PEER=$ch timeout -k 10 150 python3 scripts/bench_slab.py --ranks ${RANKS:-8,4,2} --steps 30 --rccl-self --no-check \
    > $OUT/c$ch.jsonl 2> $OUT/c$ch.err || { tail -5 $OUT/c$ch.err; exit 1; }
  fi
  python3 -c "
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print('channels', sys.argv[2], 'ranks', d['ranks'], d['ms_per_step'], d['rep_ms_per_step'])
" $OUT/c$ch.jsonl $ch
done
