#!/bin/bash
# Round 4, lease d: kernel traces of the 256^3 physical runs (free surfaces, two
# materials, no faces) and the bare 256^3 / 512^3 step, plus the fixed tests.
# Output under gpurun_out/r4/d.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/d
mkdir -p $OUT
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_engine.py tests/test_gpu_faces.py -k "time_dependent or partial_face" > $OUT/first.txt 2>&1
rc=$?; echo "first rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/first.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
tr() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "$n rc=$?"; tail -5 $OUT/$n.err; exit 1; }
  tail -1 $OUT/$n.json
  python3 - $OUT/$n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for r in list(csv.DictReader(open(f[0])))[:6]:
    print(f"  {r['Name'][:90]:90s} n {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  {float(r['Percentage']):5.1f}%")
PY
}
tr het256 python3 scripts/bench_physics.py --n 256 --layers --steps 20
tr free256 python3 scripts/bench_physics.py --n 256 --steps 20
tr nofree256 python3 scripts/bench_physics.py --n 256 --no-free --steps 20
tr hetnofree256 python3 scripts/bench_physics.py --n 256 --layers --no-free --steps 20
tr bench256 python3 bench.py --n 256 --steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-profile
timeout -k 10 200 python bench.py --n 256 --steps 20 --warmup 5 --reps 5 --no-cpu-baseline > $OUT/bench256_bare.json 2> $OUT/bench256_bare.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench256_bare.json'));r=d['roofline'];print('bare256',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['copy_ceiling']['GBps'])"
