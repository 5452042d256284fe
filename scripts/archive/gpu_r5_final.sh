#!/bin/bash
# Round 5, the ONE end-of-round lease: box characterisation,
# full GPU suite, smoke, the default bench line, bare and traced bench runs,
# 256^3 (steady: 100 steps), the RCCL self-exchange lines (whole grid and the
# N = 8 slab), the simplex lines, 512^3 physical runs, and rocprofv3 evidence
# (trace + FETCH_SIZE + WRITE_SIZE) for profiles/pmc_traffic.json of this build;
# the 2-D step lines and a 1024^3 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-final}
mkdir -p $OUT
bash scripts/box_char.sh $OUT || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -30; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('default',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['copy_ceiling']['frac_of_copy'],r['traffic'],r.get('traffic_source'))"
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline"
timeout -k 10 200 python bench.py $BA > $OUT/bare1.json 2> $OUT/bare1.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace1 -o run -- python3 bench.py $BA > $OUT/traced1.json 2> $OUT/traced1.err || exit 1
for f in bare1 traced1; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));r=d['roofline'];print('$f',d['ms_per_step'],r['kernel_avg_ms'],r['frac'])"; done
timeout -k 10 300 python bench.py --n 256 --steps 100 --warmup 20 --reps 7 --no-cpu-baseline > $OUT/bench_256.json 2> $OUT/bench_256.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_256.json'));r=d['roofline'];print('256',d['ms_per_step'],r['kernel_avg_ms'],r['frac'])"
timeout -k 10 300 python bench.py --rccl-self --steps 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_rccl_self.json 2> $OUT/bench_rccl_self.err || exit 1
timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8_rccl_self.json 2> $OUT/slab8_rccl_self.err || exit 1
tail -1 $OUT/slab8_rccl_self.json
timeout -k 10 300 python scripts/bench_simplex.py --workloads cubetask,fracture --n 16 --steps 200 > $OUT/simplex16.jsonl 2> $OUT/simplex16.err || exit 1
timeout -k 10 300 python scripts/bench_2d.py --steps 100 > $OUT/bench_2d.jsonl 2> $OUT/bench_2d.err || exit 1
cat $OUT/bench_2d.jsonl
# 1024^3 on one GPU (2 x 80 GB layers; Z = 1024: the one-plane k_fused_xyz)
timeout -k 10 400 python bench.py --n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_1024.json 2> $OUT/bench_1024.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_1024.json'));r=d['roofline'];print('1024',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel'])"
for a in "free512:--n 512 --steps 10" "het512:--n 512 --steps 10 --layers" "hetmax512:--n 512 --steps 10 --layers --maxwell"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python3 scripts/bench_physics.py $args > $OUT/phys_$n.json 2> $OUT/phys_$n.err || { echo "$n rc=$?"; exit 1; }
  tail -1 $OUT/phys_$n.json
done
TAG=${PTAG:-r5final} timeout -k 10 900 bash scripts/gpu_profile.sh > $OUT/profile.log 2>&1; echo "profile rc=$?"; tail -3 $OUT/profile.log
