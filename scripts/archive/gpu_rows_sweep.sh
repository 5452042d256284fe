#!/bin/bash
# Rows-per-block sweep of the one-pass step on one box (same library): N in $SIZES.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rows
for n in ${SIZES:-512 256}; do
  for rows in ${ROWS:-0 32 64 128 256 512}; do
    timeout -k 10 200 python bench.py --n $n --steps 20 --no-cpu-baseline --rows-per-block $rows \
      > gpurun_out/rows/n${n}_r$rows.json 2> gpurun_out/rows/n${n}_r$rows.err || exit $?
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print('n', sys.argv[2], 'rows', sys.argv[3], r['value'], r['roofline']['kernel_avg_ms'])" \
      gpurun_out/rows/n${n}_r$rows.json $n $rows
  done
done
