#!/bin/bash
# Round 6, the end-of-round lease on the final build (final5: + SIMD partners on neighbouring z blocks):
# box characterisation, the
# full GPU suite, smoke, the default bench line, 256^3 and 1024^3 lines, the RCCL
# self-exchange lines, simplex / 2-D / physics lines, and the rocprofv3 evidence
# (kernel trace + FETCH_SIZE + WRITE_SIZE at 512^3 and 256^3) from which
# profiles/pmc_traffic*.json of this build are made.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/${LEASE:-final5}
mkdir -p $OUT
bash scripts/box_char.sh $OUT || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.txt | head -30; tail -1 $OUT/pytest_gpu.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('default',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['copy_ceiling']['frac_of_copy'],d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --n 256 --steps 100 --warmup 20 --reps 7 --no-cpu-baseline > $OUT/bench_256.json 2> $OUT/bench_256.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_256.json'));r=d['roofline'];print('256',d['ms_per_step'],r['kernel_avg_ms'],r['frac'])"
timeout -k 10 400 python bench.py --n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_1024.json 2> $OUT/bench_1024.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_1024.json'));r=d['roofline'];print('1024',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel_symbol'])"
timeout -k 10 300 python bench.py --rccl-self --steps 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_rccl_self.json 2> $OUT/bench_rccl_self.err || exit 1
timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8_rccl_self.json 2> $OUT/slab8_rccl_self.err || exit 1
tail -1 $OUT/slab8_rccl_self.json | cut -c1-400
timeout -k 10 300 python scripts/bench_slab.py --ranks 8 --loop-gbps 64 --no-check > $OUT/slab8_loop64.json 2> $OUT/slab8_loop64.err || exit 1
timeout -k 10 300 python scripts/bench_simplex.py --workloads cubetask,fracture --n 16 --steps 200 > $OUT/simplex16.jsonl 2> $OUT/simplex16.err || exit 1
timeout -k 10 300 python scripts/bench_2d.py --steps 100 > $OUT/bench_2d.jsonl 2> $OUT/bench_2d.err || exit 1
for a in "free512:--n 512 --steps 10" "het512:--n 512 --steps 10 --layers" "hetmax512:--n 512 --steps 10 --layers --maxwell"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python3 scripts/bench_physics.py $args > $OUT/phys_$n.json 2> $OUT/phys_$n.err || { echo "$n rc=$?"; exit 1; }
done
TAG=r6final5_512 timeout -k 10 600 bash scripts/gpu_profile.sh > $OUT/profile512.log 2>&1; echo "profile 512 rc=$?"; tail -2 $OUT/profile512.log
N=256 STEPS=100 TAG=r6final5_256 timeout -k 10 600 bash scripts/gpu_profile.sh > $OUT/profile256.log 2>&1; echo "profile 256 rc=$?"; tail -2 $OUT/profile256.log
N=1024 STEPS=3 TAG=r6final5_1024 timeout -k 10 600 bash scripts/gpu_profile.sh > $OUT/profile1024.log 2>&1; echo "profile 1024 rc=$?"; tail -2 $OUT/profile1024.log
