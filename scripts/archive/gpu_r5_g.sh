#!/bin/bash
# Round 5, lease G: box characterisation, then A/B of the prologue pipelining
# (current build) against the previous Lagrange build (tune/lag), 256^3 steady
# (100 steps) and 512^3, alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-g}
mkdir -p $OUT
bash scripts/box_char.sh $OUT || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fma.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline']
print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'])" "$1" "$2"; }
for rep in 1 2 3; do
  for v in lag cur; do
    if [ $v = lag ]; then L=gcm_amd/lib/tune/lag/libgcmx.so; else L=gcm_amd/lib/libgcmx.so; fi
    GCMX_LIB=$L timeout -k 10 200 python bench.py --n 256 --steps 100 --warmup 20 --reps 5 --no-cpu-baseline --no-copy-ceiling --no-box-state > $OUT/ab_${v}_256_$rep.json 2> $OUT/ab_${v}_256_$rep.err || { echo "rc=$?"; exit 1; }
    summ $OUT/ab_${v}_256_$rep.json "$v 256 rep$rep"
    GCMX_LIB=$L timeout -k 10 200 python bench.py --n 512 --steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling --no-box-state > $OUT/ab_${v}_512_$rep.json 2> $OUT/ab_${v}_512_$rep.err || { echo "rc=$?"; exit 1; }
    summ $OUT/ab_${v}_512_$rep.json "$v 512 rep$rep"
  done
done
