#!/bin/bash
# Round 4, final lease: full GPU suite, the default bench line, bare/traced
# alternation on one box, 256^3 bench, 512^3 physical runs, and rocprofv3
# evidence (trace + FETCH/WRITE) for profiles/pmc_traffic.json of this build.
# Output under gpurun_out/r4/final and gpurun_out/prof_r4final.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/${LEASE:-final}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -30; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('default',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['copy_ceiling']['frac_of_copy'],r['traffic'],r.get('traffic_source'))"
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 200 python bench.py $BA > $OUT/bare$i.json 2> $OUT/bare$i.err || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$i -o run -- python3 bench.py $BA > $OUT/traced$i.json 2> $OUT/traced$i.err || exit 1
  for f in bare$i traced$i; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));r=d['roofline'];print('$f',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],d['process_state']['clock']['mhz_median'])"; done
done
timeout -k 10 200 python bench.py --n 256 $BA > $OUT/bench_256.json 2> $OUT/bench_256.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_256.json'));r=d['roofline'];print('256',d['ms_per_step'],r['kernel_avg_ms'],r['frac'])"
for a in "free512:--n 512 --steps 10" "het512:--n 512 --steps 10 --layers" "hetmax512:--n 512 --steps 10 --layers --maxwell"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python3 scripts/bench_physics.py $args > $OUT/phys_$n.json 2> $OUT/phys_$n.err || { echo "$n rc=$?"; exit 1; }
  tail -1 $OUT/phys_$n.json
done
TAG=${PTAG:-r4final} timeout -k 10 900 bash scripts/gpu_profile.sh > $OUT/profile.log 2>&1; echo "profile rc=$?"; tail -3 $OUT/profile.log
