#!/bin/bash
# Same-box A/B of the two floating-point builds of the 512^3 step (bench.py,
# GCMX_FP=exact vs the FMA default), alternating, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for fp in exact fma; do
    GCMX_FP=$fp timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$fp', d['ms_per_step'], r['kernel_avg_ms'], r['frac'], r['kernel_symbol'], 'copy', r['copy_ceiling']['GBps'])" || exit 1
  done
done
