#!/bin/bash
# NB kernel: phase timers, rows-per-block sweep (tuning builds under gcm_amd/lib/tune).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nb
T=gcm_amd/lib/tune
GCMX_LIB=$T/diag/libgcmx.so timeout -k 10 120 python scripts/tx2_diag.py > gpurun_out/nb/diag.txt 2>&1 || exit $?
cat gpurun_out/nb/diag.txt
for rows in 128 256 512 64; do
  GCMX_LIB=$T/nb/libgcmx.so timeout -k 10 200 python bench.py --n 512 --steps 20 --no-cpu-baseline \
    --rows-per-block $rows > gpurun_out/nb/rows_$rows.json 2> gpurun_out/nb/rows_$rows.err || exit $?
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['value'], r['roofline']['kernel_avg_ms'])" gpurun_out/nb/rows_$rows.json $rows
done
