#!/bin/bash
# Round 4: alternating-direction y march -- parity suites first, then A/B timing
# (alt vs noalt) at 512^3, 256^3 and a 64-plane 512^2 slab emulation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/${LEASE:-alt}
mkdir -p $OUT gpurun_out/ab
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_faces.py \
  tests/test_gpu_fma.py tests/test_gpu_slabs.py tests/test_gpu_engine.py -m gpu > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -30; tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_run.sh > $OUT/ab512.txt 2>&1 && N=256 bash scripts/ab_run.sh > $OUT/ab256.txt 2>&1
cat $OUT/ab512.txt $OUT/ab256.txt
for v in alt noalt; do
  GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so timeout -k 10 200 python bench.py --emulate-slabs 8 --steps 10 --reps 3 > $OUT/emu8_$v.json 2> $OUT/emu8_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/emu8_$v.json'));print('emu8 $v',d['ms_per_step'],d.get('value'))"
done
