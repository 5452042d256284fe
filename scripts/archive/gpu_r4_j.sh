#!/bin/bash
# Round 4, lease j: rates of this round's engine paths at 256^3 -- partial faces
# (per-node face maps), bodies stacked along x / y / z with contacts (y / z: one
# stack grid), against one body.  Output under gpurun_out/r4/j.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/${LEASE:-j}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_faces.py tests/test_gpu_engine.py tests/test_gpu_fma.py -m gpu > $OUT/pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
for a in "one:--no-free" "free:" "partial:--partial" "x4:--xbodies 4 --axis 0" "y4:--xbodies 4 --axis 1" "z4:--xbodies 4 --axis 2" \
         "y4nostack:--xbodies 4 --axis 1 NOSTACK" "partialmaps0:--partial NOMAPS"; do
  n=${a%%:*}; args=${a#*:}
  envs=""
  case "$args" in *NOSTACK*) envs="GCMX_NO_STACKS=1"; args=${args% NOSTACK};; esac
  case "$args" in *NOMAPS*) envs="GCMX_NO_FACE_MAPS=1"; args=${args% NOMAPS};; esac
  if [ -n "$envs" ]; then export $envs; fi
  timeout -k 10 200 python3 scripts/bench_physics.py --n 256 --steps 30 $args > $OUT/phys_$n.json 2> $OUT/phys_$n.err || { echo "$n rc=$?"; tail -3 $OUT/phys_$n.err; exit 1; }
  unset GCMX_NO_STACKS GCMX_NO_FACE_MAPS
  python3 -c "import json;d=json.load(open('$OUT/phys_$n.json'));print('$n',d['ms_per_step'],d['last_path'],d['metric'])"
done
