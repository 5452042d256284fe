#!/bin/bash
# Slab-schedule timing on one GPU (scripts/bench_slab.py) under several settings,
# then the GPU parity suite with the slab schedule forced on every fused step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/slab
run() {  # $1 = tag, rest = env assignments
  tag=$1; shift
  env "$@" timeout -k 10 300 python scripts/bench_slab.py > gpurun_out/slab/$tag.jsonl 2> gpurun_out/slab/$tag.err
  rc=$?; echo "== $tag rc=$rc"; cat gpurun_out/slab/$tag.jsonl
  [ $rc -eq 0 ] || { tail -5 gpurun_out/slab/$tag.err; exit $rc; }
}
run unsplit GCMX_SLAB_SCHEDULE=0
run old_onestream GCMX_SLAB_SCHEDULE=2
run split GCMX_SLAB_SCHEDULE=1
GCMX_SLAB_SCHEDULE=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/slab/pytest_split.log 2>&1
rc=$?; echo "pytest (slab schedule forced) rc=$rc"; tail -3 gpurun_out/slab/pytest_split.log; exit $rc
