#!/bin/bash
# Round 5, lease D: the HET / FMA / parity suites on the build without the
# waterfall, and 256^3 at steady state (longer runs: does
# the short default run see a lower clock?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fma.py tests/test_gpu_faces.py -m gpu -q --timeout 300 --timeout-method thread -k "heterogeneous or het or HET or layers" > $OUT/pytest_het.txt 2>&1
rc=$?; echo "pytest het rc=$rc"; tail -3 $OUT/pytest_het.txt
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c "
import json,sys,statistics;d=json.load(open(sys.argv[1]));r=d['roofline'];b=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (b.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'],'power',b.get('power_w'),'sclk',statistics.median(sc) if sc else None)" "$1" "$2"; }
for st in 20 100 400; do
  timeout -k 10 300 python bench.py --n 256 --steps $st --warmup 50 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b256_s$st.json 2> $OUT/b256_s$st.err || { echo "rc=$?"; exit 1; }
  summ $OUT/b256_s$st.json "256 steps $st"
done
timeout -k 10 300 python bench.py --n 256 --steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b256_short.json 2> $OUT/b256_short.err && summ $OUT/b256_short.json "256 short (warmup 5)"
# A/B: the shipped build against the tuning variants under gcm_amd/lib/tune (except base)
BA="--steps 20 --warmup 20 --reps 5 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2; do
  for d in gcm_amd/lib gcm_amd/lib/tune/unroll5; do
    [ -f $d/libgcmx.so ] || continue
    v=$(basename $d)
    for n in 512 256; do
      GCMX_LIB=$d/libgcmx.so timeout -k 10 200 python bench.py --n $n $BA > $OUT/ab_${v}_${n}_$rep.json 2> $OUT/ab_${v}_${n}_$rep.err || { echo "ab $v $n rc=$?"; tail -3 $OUT/ab_${v}_${n}_$rep.err; exit 1; }
      summ $OUT/ab_${v}_${n}_$rep.json "$v $n rep$rep"
    done
  done
done
