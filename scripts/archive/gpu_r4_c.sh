#!/bin/bash
# Round 4, lease c: the run-b failures first (end-of-step post rule, plain HET
# table loads, test fixes), then the touched suites without -x, the x-marching
# probe, the 256^3 HET / free-surface steps and the default bench.
# Output under gpurun_out/r4/c.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/c
mkdir -p $OUT
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_slabs.py tests/test_gpu_fma.py tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_faces.py \
  -k "mixed_material_ids or heterogeneous or xbodies or step_ode or stack or partial_face or time_dependent" > $OUT/first.txt 2>&1
rc=$?; echo "first rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/first.txt | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 1000 $PT tests/test_gpu_fma.py tests/test_gpu_slabs.py tests/test_gpu_parity.py \
  tests/test_gpu_engine.py tests/test_gpu_faces.py -m gpu > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -40; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
XM_ONLY=1 timeout -k 10 120 ./tools/xyz_probe > $OUT/xyz_probe_xm.txt 2>&1; echo "probe rc=$?"; cat $OUT/xyz_probe_xm.txt
timeout -k 10 200 python scripts/bench_physics.py --n 256 --layers --steps 20 > $OUT/het256.json 2> $OUT/het256.err; echo "het rc=$?"; cat $OUT/het256.json
timeout -k 10 200 python scripts/bench_physics.py --n 256 --steps 20 > $OUT/free256.json 2> $OUT/free256.err; echo "free rc=$?"; cat $OUT/free256.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --reps 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['ms_per_step'],r['kernel_avg_ms'],r['frac'],d['process_state']['clock'])"
