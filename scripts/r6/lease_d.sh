#!/bin/bash
# Round 6, lease D: where the 1024^3 z-split step's time goes -- rocprofv3
# kernel trace (k_step_tx2 ZS and k_zseam separately), rows per block 256 / 512 /
# 1024 (automatic), 64 MiB physical chunks; the FMA Z = 1024 tolerance case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/d
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_fma.py -k "sizes6" > $OUT/pytest_fma1024.txt 2>&1
echo "fma-1024 rc=$?"; tail -1 $OUT/pytest_fma1024.txt
BA="--n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1024 -o run -- python3 bench.py $BA > $OUT/traced_1024.json 2> $OUT/traced_1024.err || { echo "trace rc=$?"; tail -3 $OUT/traced_1024.err; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$OUT/trace1024/run_kernel_stats.csv")))
for r in rows[:6]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"])/1e6, 4), "ms")
PY
for v in "r256:--rows-per-block 256" "r512:--rows-per-block 512" "auto:" "c64:GCMX_ALLOC=shuffle:64"; do
  tag=${v%%:*}; arg=${v#*:}
  if [[ $arg == GCMX_* ]]; then envs=$arg; arg=""; else envs=""; fi
  env $envs timeout -k 10 400 python bench.py $BA $arg > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b_$tag.json'));r=d['roofline'];print('$tag',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],d['process_state']['layers']['alloc'])"
done
