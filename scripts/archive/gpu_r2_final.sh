#!/bin/bash
# r2 evidence for the shipped one-pass step: kernel trace + FETCH/WRITE + SQ passes
# (gpu_profile.sh), counter passes (gpu_counters.sh), 256^3 bench, free-surface
# physics bench at 512^3.  Output under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2nb}
TAG=$TAG SQ=1 bash scripts/gpu_profile.sh || exit $?
TAG=$TAG bash scripts/gpu_counters.sh || exit $?
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --n 256 > gpurun_out/$TAG/bench_256.json 2> gpurun_out/$TAG/bench_256.err || exit $?
timeout -k 10 300 python scripts/bench_physics.py --n 512 > gpurun_out/$TAG/physics_512.json 2> gpurun_out/$TAG/physics_512.err || exit $?
cat gpurun_out/$TAG/physics_512.json
