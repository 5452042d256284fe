#!/bin/bash
# Round 6, lease F: the z split at Z = 512 (GCMX_ZS_PART=256: each 512-node row
# as two independent 256-lane blocks of 4 waves, 2 blocks per CU, cut Z stages
# by k_zseam) against the one-block-per-row step: parity first, then 512^3
# alternating A/B over rows per block.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/f
mkdir -p $OUT
GCMX_ZS_PART=256 timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fused_step_3d or zsplit or full_size_512 or uni_instance" > $OUT/pytest_zs256.txt 2>&1
rc=$?; echo "zs256 parity rc=$rc"; tail -1 $OUT/pytest_zs256.txt; [ $rc -eq 0 ] || exit 1
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2; do
  for v in "base::" "zs256r512:GCMX_ZS_PART=256:--rows-per-block 512" "zs256r128:GCMX_ZS_PART=256:--rows-per-block 128" "zs256r256:GCMX_ZS_PART=256:--rows-per-block 256"; do
    tag=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; arg=${rest#*:}
    env $envs timeout -k 10 200 python bench.py $BA $arg > $OUT/b_${tag}_$rep.json 2> $OUT/b_${tag}_$rep.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_${tag}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${tag}_$rep.json'));r=d['roofline'];print('$tag $rep',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel_symbol'])"
  done
done
