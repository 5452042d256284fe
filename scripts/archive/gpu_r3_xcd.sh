#!/bin/bash
# Same-box A/B of the XCD-contiguous block order for grids whose block count is
# not a multiple of 8 (previous build in gcm_amd/lib/ab_prev): per-rank slab
# steps without exchange, twice alternating; then the automatic RCCL channel
# choice per slab size (one process each) and the slab GPU tests on the new
# build.  Output under gpurun_out/r3/xcd.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/xcd
mkdir -p $OUT
set -o pipefail
for round in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then L=gcm_amd/lib/ab_prev/libgcmx.so; else L=gcm_amd/lib/libgcmx.so; fi
    GCMX_LIB=$L timeout -k 10 150 python3 scripts/bench_slab.py --ranks 2,4,8 --steps 20 --no-check \
      > $OUT/slab_${v}_$round.jsonl 2> $OUT/slab.err || { tail -5 $OUT/slab.err; exit 1; }
    python3 -c "
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(sys.argv[2], 'ranks', d['ranks'], d['ms_per_step'], d['kernels'])
" $OUT/slab_${v}_$round.jsonl $v
  done
done
CHS=auto bash scripts/gpu_r3_rcclch.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_slabs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_slabs.log 2>&1 || { tail -20 $OUT/pytest_slabs.log; exit 1; }
tail -2 $OUT/pytest_slabs.log
