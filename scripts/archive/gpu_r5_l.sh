#!/bin/bash
# Round 5, lease L: the one-pass kernels address each block's planes from its
# own plane (grids beyond 4 GB per component plane): full GPU suite incl. the
# 82 GB probe test, A/B against the previous build (tune/prev) at 512^3 and
# 256^3, alternating, and a 1024^3 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-l}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest.txt | head -20; exit $rc; }
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline']
print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'])" "$1" "$2"; }
for rep in 1 2; do
  for v in prev cur; do
    for n in 512 256; do
      if [ $v = prev ]; then L=gcm_amd/lib/tune/prev/libgcmx.so; else L=gcm_amd/lib/libgcmx.so; fi
      GCMX_LIB=$L timeout -k 10 200 python bench.py --n $n $BA > $OUT/ab_${v}_${n}_$rep.json 2> $OUT/ab_${v}_${n}_$rep.err || { echo "ab $v $n rc=$?"; tail -3 $OUT/ab_${v}_${n}_$rep.err; exit 1; }
      summ $OUT/ab_${v}_${n}_$rep.json "$v $n rep$rep"
    done
  done
done
timeout -k 10 400 python bench.py --n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_1024.json 2> $OUT/bench_1024.err || { echo "1024 rc=$?"; tail -5 $OUT/bench_1024.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_1024.json'));r=d['roofline'];print('1024',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel'],d['value'])"
