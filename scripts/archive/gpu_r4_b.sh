#!/bin/bash
# Round 4, lease b: the HET FMA failure A/B (readfirstlane tables vs plain loads),
# then the touched GPU suites without -x (every failure in one lease), then the
# default bench (one layer allocation) twice.  Output under gpurun_out/r4/b.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/b
mkdir -p $OUT
T="tests/test_gpu_fma.py::test_fma_heterogeneous_within_tolerance tests/test_gpu_parity.py -k heterogeneous"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fma.py -k heterogeneous -v --timeout 120 --timeout-method thread > $OUT/het_rfl.txt 2>&1; echo "het rfl rc=$?"
GCMX_LIB=gcm_amd/lib/tune/norfl/libgcmx.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fma.py -k heterogeneous -v --timeout 120 --timeout-method thread > $OUT/het_norfl.txt 2>&1; echo "het norfl rc=$?"
tail -3 $OUT/het_rfl.txt $OUT/het_norfl.txt
timeout -k 10 1100 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_slabs.py tests/test_gpu_simplex.py tests/test_gpu_parity.py \
  tests/test_gpu_engine.py tests/test_gpu_faces.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest.txt | head -40; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --reps 5 --no-cpu-baseline > $OUT/bench$i.json 2> $OUT/bench$i.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench$i.json'));r=d['roofline'];print(d['ms_per_step'],r['kernel_avg_ms'],r['frac'],d['process_state']['layers']['one_allocation'],d['process_state']['clock'])"
done
# x-marching access-pattern probe beside the copy and the 2-plane pattern
XM_ONLY=1 timeout -k 10 120 ./tools/xyz_probe > $OUT/xyz_probe_xm.txt 2>&1; echo "probe rc=$?"; cat $OUT/xyz_probe_xm.txt
# heterogeneous one-pass step at 256^3 (two materials, free surfaces), the verdict's 0.85 ms
timeout -k 10 200 python scripts/bench_physics.py --n 256 --layers --steps 20 > $OUT/het256.json 2> $OUT/het256.err; cat $OUT/het256.json
timeout -k 10 200 python scripts/bench_physics.py --n 256 --steps 20 > $OUT/free256.json 2> $OUT/free256.err; cat $OUT/free256.json
