#!/bin/bash
# Same-box A/B of the tuning builds under gcm_amd/lib/tune: 512^3 and 256^3
# bench lines and the N = 8 per-rank slab step, two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abm; mkdir -p $OUT
for rep in 1 2; do
for d in gcm_amd/lib/tune/*/; do
  name=$(basename "$d")
  if [ $rep = 1 ]; then
    GCMX_FP=exact GCMX_LIB="$d/libgcmx.so" timeout -k 10 120 python scripts/ab_check.py > $OUT/$name.check 2>&1
    rc=$?; echo "$name: $(tail -1 $OUT/$name.check)"; [ $rc -le 1 ] || exit $rc
  fi
  r512=$(GCMX_LIB="$d/libgcmx.so" timeout -k 10 200 python bench.py --n 512 --steps 20 --no-cpu-baseline --no-copy-ceiling 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['roofline']['kernel_avg_ms'])") || exit 1
  r256=$(GCMX_LIB="$d/libgcmx.so" timeout -k 10 200 python bench.py --n 256 --steps 40 --no-cpu-baseline --no-copy-ceiling 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['roofline']['kernel_avg_ms'])") || exit 1
  rs=$(GCMX_LIB="$d/libgcmx.so" timeout -k 10 200 python scripts/bench_slab.py --ranks 8 --steps 30 --no-check 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'): d=json.loads(l); print(d['ms_per_step'], d['kernels'].get('fused_xyz_boundary'))") || exit 1
  echo "$name rep $rep: 512^3 $r512 ms  256^3 $r256 ms  N=8 slab $rs"
done
done
