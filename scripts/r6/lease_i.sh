#!/bin/bash
# Round 6, lease I: the z split with the cut columns recomputed by k_zseam (no
# hand-over through memory): parity, then shapes and the 1024^3 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_fma.py -k "zsplit or sizes6" > $OUT/pytest_zs.txt 2>&1
rc=$?; echo "zsplit parity rc=$rc"; tail -1 $OUT/pytest_zs.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_zs.txt | head; exit 1; }
GCMX_ZS_PART=256 timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fused_step_3d or zsplit or full_size_512" > $OUT/pytest_zs256.txt 2>&1
rc=$?; echo "zs256 parity rc=$rc"; tail -1 $OUT/pytest_zs256.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/bench_shape.py 512,512,1024 1024,1024,512 512,512,512 > $OUT/shapes.jsonl 2> $OUT/shapes.err || { echo "shapes rc=$?"; tail -3 $OUT/shapes.err; exit 1; }
cut -c1-170 $OUT/shapes.jsonl
GCMX_ZS_PART=256 timeout -k 10 300 python scripts/bench_shape.py 512,512,512 > $OUT/shapes_zs256.jsonl 2> $OUT/shapes_zs256.err || { echo "zs256 rc=$?"; exit 1; }
cut -c1-170 $OUT/shapes_zs256.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1024 -o run -- python3 bench.py --n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_1024.json 2> $OUT/bench_1024.err || { echo "bench 1024 rc=$?"; tail -3 $OUT/bench_1024.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_1024.json'));r=d['roofline'];print('1024',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel_symbol'])"
python3 - <<PY
import csv
for r in list(csv.DictReader(open("$OUT/trace1024/run_kernel_stats.csv")))[:5]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"])/1e6, 4), "ms")
PY
