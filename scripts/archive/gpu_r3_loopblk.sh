#!/bin/bash
# Loopback exchange: sensitivity of one rank's step to the transfer's CU
# footprint (blocks of the copy kernel) at 64 GB/s per direction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/${TAG:-loopblk}
mkdir -p $OUT
set -o pipefail
for B in ${BLOCKS:-8 32 64 128}; do
  timeout -k 10 200 python scripts/bench_slab.py --loop-gbps ${RATE:-64} --loop-blocks $B --ranks 8,4 --steps 30 --no-check \
    >> $OUT/slab_loop.jsonl 2>> $OUT/slab.err || { echo "bench_slab rc=$?"; tail $OUT/slab.err; exit 1; }
done
python - <<'PY' $OUT
import json, sys
for l in open(sys.argv[1] + "/slab_loop.jsonl"):
    d = json.loads(l)
    print(d["exchange"], d["ranks"], d["ms_per_step"], d["kernels"])
PY
