#!/bin/bash
# Round 5, lease M: steady-state 256^3 A/B (100-step repetitions) of the
# per-block plane bases against the previous build, alternating, three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-m}
mkdir -p $OUT
BA="--n 256 --steps 100 --warmup 20 --reps 7 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2 3; do
  for v in cur prev; do
    if [ $v = prev ]; then L=gcm_amd/lib/tune/prev/libgcmx.so; else L=gcm_amd/lib/libgcmx.so; fi
    GCMX_LIB=$L timeout -k 10 200 python bench.py $BA > $OUT/s256_${v}_$rep.json 2> $OUT/s256_${v}_$rep.err || { echo "$v rc=$?"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'])" $OUT/s256_${v}_$rep.json "$v rep$rep"
  done
done
