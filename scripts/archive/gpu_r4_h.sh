#!/bin/bash
# Round 4, lease h: the full GPU suite, the default bench line, 256^3 bench,
# the 256^3 physical runs under a kernel trace, then rocprofv3 evidence for the
# 512^3 bench (trace + FETCH/WRITE + SQ passes).  Output under gpurun_out/r4/h
# and gpurun_out/prof_r4h.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/h
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -30; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('default',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['copy_ceiling']['frac_of_copy'],d['cpu_baseline'])"
timeout -k 10 200 python bench.py --n 256 --steps 20 --warmup 5 --reps 5 --no-cpu-baseline > $OUT/bench_256.json 2> $OUT/bench_256.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_256.json'));r=d['roofline'];print('256',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['copy_ceiling']['frac_of_copy'])"
for a in "het:--layers" "free:" "hetnofree:--layers --no-free" "nofree:--no-free" "hetmax:--layers --maxwell"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/phys_$n -o run -- python3 scripts/bench_physics.py --n 256 --steps 30 $args > $OUT/phys_$n.json 2> $OUT/phys_$n.err || { echo "$n rc=$?"; exit 1; }
  tail -1 $OUT/phys_$n.json
done
TAG=r4h SQ=1 timeout -k 10 900 bash scripts/gpu_profile.sh > $OUT/profile.log 2>&1; echo "profile rc=$?"; tail -5 $OUT/profile.log
