#!/bin/bash
# Round 5, lease C: full GPU suite on the Lagrange-form FMA build, A/B of the
# round-4 build (tune/base) against it at 512^3 and 256^3 (alternating, one
# box), a long 512^3 bench for steady power, the simplex lines with the launch
# floor and the per-mesh fusion choice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-c}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest.txt | head -20; exit $rc; }
fi
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];b=d['process_state'].get('box_during_reps') or {}
print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'],'power',b.get('power_w'))" "$1" "$2"; }
for rep in 1 2; do
  for v in base cur; do
    for n in 512 256; do
      if [ $v = base ]; then L=gcm_amd/lib/tune/base/libgcmx.so; else L=gcm_amd/lib/libgcmx.so; fi
      GCMX_LIB=$L timeout -k 10 200 python bench.py --n $n $BA > $OUT/ab_${v}_${n}_$rep.json 2> $OUT/ab_${v}_${n}_$rep.err || { echo "ab $v $n rc=$?"; tail -3 $OUT/ab_${v}_${n}_$rep.err; exit 1; }
      summ $OUT/ab_${v}_${n}_$rep.json "$v $n rep$rep"
    done
  done
done
timeout -k 10 300 python bench.py --steps 100 --reps 7 --no-cpu-baseline > $OUT/bench_long.json 2> $OUT/bench_long.err || { echo "bench rc=$?"; tail -5 $OUT/bench_long.err; exit 1; }
summ $OUT/bench_long.json long512
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
summ $OUT/bench_default.json default
timeout -k 10 300 python scripts/bench_simplex.py --workloads cubetask,fracture --n 16 --steps 200 > $OUT/simplex16.jsonl 2> $OUT/simplex16.err || { echo "simplex rc=$?"; tail -5 $OUT/simplex16.err; exit 1; }
cat $OUT/simplex16.jsonl
for f in 1 2; do
  timeout -k 10 300 python scripts/bench_simplex.py --workloads cubetask,fracture --n 16 --steps 200 --fusion $f > $OUT/simplex16_f$f.jsonl 2>> $OUT/simplex16.err || { echo "simplex f$f rc=$?"; exit 1; }
  python3 -c "import json;[print('fusion $f', d['workload'], d['ms_per_step'], d['launches_per_step']) for d in map(json.loads, open('$OUT/simplex16_f$f.jsonl'))]"
done
