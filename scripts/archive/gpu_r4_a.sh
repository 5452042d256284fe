#!/bin/bash
# Round 4, first lease: the swing probe (scripts/swing_probe.sh), then the GPU
# tests touched by global x-pairing, the one-post-per-step rule and the new
# FMA engine tests.  Output under gpurun_out/r4/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-a} bash scripts/swing_probe.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_slabs.py tests/test_gpu_simplex.py tests/test_gpu_parity.py \
  tests/test_gpu_engine.py tests/test_gpu_faces.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_a.txt 2>&1
rc=$?; tail -5 gpurun_out/r4/pytest_a.txt; exit $rc
