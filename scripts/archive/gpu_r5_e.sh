#!/bin/bash
# Round 5, lease E: box characterisation, then the 256^3 PMC read ratio of the
# current build (trace + FETCH_SIZE + WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/box_char.sh gpurun_out/r5/e || exit 1
N=256 STEPS=20 TAG=r5e256 timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/r5/e/profile256.log 2>&1; rc=$?; echo "profile rc=$rc"; tail -3 gpurun_out/r5/e/profile256.log
