#!/bin/bash
# Same-box A/B of the simplex kernels: the current libgcmx.so against the one
# under gcm_amd/lib/sxold (loaded through LD_LIBRARY_PATH / GCMX_LIB), one
# thread per node at 64^3 and the automatic layout at 16^3 / 32^3; then the
# simplex GPU tests on the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/${TAG:-sxab}
mkdir -p $OUT
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_simplex.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export LD_LIBRARY_PATH=$PWD/gcm_amd/lib/sxold GCMX_LIB=$PWD/gcm_amd/lib/sxold/libgcmx.so; else unset LD_LIBRARY_PATH GCMX_LIB; fi
    timeout -k 10 200 python scripts/bench_simplex.py --workloads cube,fracture,layered --n 64 --lanes 1 --steps 20 \
      | sed "s/^/$v /" >> $OUT/ab64.txt || exit 1
    timeout -k 10 200 python scripts/bench_simplex.py --workloads cube,cubetask --n 32 --steps 100 \
      | sed "s/^/$v /" >> $OUT/ab32.txt || exit 1
  done
done
unset LD_LIBRARY_PATH GCMX_LIB
python3 - <<'PY' $OUT
import json, sys
for f in ("ab64.txt", "ab32.txt"):
    for l in open(sys.argv[1] + "/" + f):
        v, j = l.split(" ", 1)
        d = json.loads(j)
        print(f, v, d["workload"], d["vertices"], d["ms_per_step"], d["value"])
PY
