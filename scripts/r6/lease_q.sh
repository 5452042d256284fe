#!/bin/bash
# Round 6 lease Q: borderSize 3 on the one-pass path -- k_fused_xyz<3, ...> at
# 2 waves per SIMD (no spills) against the round-5 occupancy 4 (97 VGPRs
# spilled; tune build gcm_amd/lib/tune/bs3mw4), the bs = 3 parity cases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/q
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fma.py > $OUT/pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 1 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export GCMX_LIB=gcm_amd/lib/tune/bs3mw4/libgcmx.so; else unset GCMX_LIB; fi
    timeout -k 10 200 python scripts/bench_shape.py 512,512,512 256,256,256 512,512,1024 --bs 3 --steps 5 --reps 3 > $OUT/bs3_${v}_$i.jsonl 2> $OUT/bs3_${v}_$i.err || { echo "$v rc=$?"; exit 1; }
    echo "$v $i"; cut -c1-200 $OUT/bs3_${v}_$i.jsonl
  done
done
unset GCMX_LIB
timeout -k 10 200 python scripts/bench_shape.py 512,512,512 --steps 5 --reps 3 > $OUT/bs2.jsonl 2>&1 && cut -c1-200 $OUT/bs2.jsonl
