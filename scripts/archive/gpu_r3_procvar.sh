#!/bin/bash
# Per-process spread of the 512^3 step on one box: 5 fresh bench processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('proc', $i, d['ms_per_step'], r['kernel_avg_ms'], 'copy', r['copy_ceiling']['GBps'])" || exit 1
done
