#!/bin/bash
# Round-3: one rank's step with the exchange in flight (loopback transport at
# emulated xGMI rates) for the boundary-first and X-slab schedules, and the
# loopback parity tests.  Output under gpurun_out/r3/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/${TAG:-loop}
mkdir -p $OUT
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_slabs.py -m gpu -x -v -k "loopback or local_group_fused or rccl" \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for G in ${RATES:-0 50 64}; do
  for S in bfirst xslab; do
    timeout -k 10 200 python scripts/bench_slab.py --sched $S --loop-gbps $G --ranks 8,4,2 --steps 30 --no-check \
      >> $OUT/slab_loop.jsonl 2>> $OUT/slab.err || { echo "bench_slab rc=$?"; tail $OUT/slab.err; exit 1; }
  done
done
timeout -k 10 200 python scripts/bench_slab.py --ranks 8,4,2 --steps 30 --no-check >> $OUT/slab_noexchange.jsonl 2>> $OUT/slab.err || exit 1
python - <<'EOF' $OUT
import json, sys
for f in ("slab_loop.jsonl", "slab_noexchange.jsonl"):
    for l in open(sys.argv[1] + "/" + f):
        d = json.loads(l)
        print(d["sched"], d["exchange"][:30], d["ranks"], d["ms_per_step"], d["kernel_ms_per_step"], d["kernels"])
EOF
