#!/bin/bash
# Round 5, lease A: full GPU suite on the med3-limiter build, A/B of the
# shipped round-4 build (tune/base) against it at 512^3 and 256^3 (alternating,
# one box), the default bench line with the box state, and the four-planes /
# one-wave-per-SIMD access-pattern probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'])" "$1" "$2"; }
for rep in 1 2; do
  for v in base cur; do
    for n in 512 256; do
      if [ $v = base ]; then L=gcm_amd/lib/tune/base/libgcmx.so; else L=gcm_amd/lib/libgcmx.so; fi
      GCMX_LIB=$L timeout -k 10 200 python bench.py --n $n $BA > $OUT/ab_${v}_${n}_$rep.json 2> $OUT/ab_${v}_${n}_$rep.err || { echo "ab $v $n rc=$?"; tail -3 $OUT/ab_${v}_${n}_$rep.err; exit 1; }
      summ $OUT/ab_${v}_${n}_$rep.json "$v $n rep$rep"
    done
  done
done
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench rc=$?"; tail -5 $OUT/bench_default.err; exit 1; }
summ $OUT/bench_default.json default
timeout -k 10 120 env TX4_ONLY=1 ./tools/xyz_probe > $OUT/xyz_probe_tx4.txt 2>&1; echo "probe rc=$?"; cat $OUT/xyz_probe_tx4.txt
