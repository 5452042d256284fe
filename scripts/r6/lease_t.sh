#!/bin/bash
# Round 6 lease T: the two-generation split on by default (64 %): its parity
# tests, then 256^3 on / off alternating, 512^3 unchanged.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6/t
mkdir -p $OUT
for st in fresh after_import after_ctx torch_first; do timeout -k 10 120 python scripts/r6/probe_torch.py $st 2>&1 | tail -n 6; done
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "two_generation or full_size_256 or heterogeneous_one_pass" > $OUT/pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 1 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 0 64; do
    GCMX_TX2_GEN2=$v timeout -k 10 120 python scripts/bench_shape.py 256,256,256 --steps 20 --reps 5 > $OUT/g${v}_$i.json 2> $OUT/g${v}_$i.err || { echo "$v rc=$?"; exit 1; }
    echo "$v $i $(cut -c1-160 $OUT/g${v}_$i.json)"
  done
done
timeout -k 10 120 python scripts/bench_shape.py 512,512,512 --steps 5 --reps 3 | cut -c1-200
