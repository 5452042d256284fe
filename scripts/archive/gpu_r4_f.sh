#!/bin/bash
# Round 4, lease f: HET table source (LDS vs scalar loads), skipped last X row,
# restructured face ghosts: parity of the variants' HET paths, then 256^3 wall
# time per step.  Output under gpurun_out/r4/f.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/${LEASE:-f}
mkdir -p $OUT
for v in new3; do
  GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so LD_LIBRARY_PATH=gcm_amd/lib/tune/$v timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_fma.py tests/test_gpu_faces.py -k "heterogeneous or face_map or partial" > $OUT/pytest_$v.txt 2>&1
  rc=$?; echo "$v pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_$v.txt | tail -6
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
run() {  # variant, label, args...
  local v=$1 l=$2; shift 2
  local lp=""
  [ "$v" = base ] || lp=gcm_amd/lib/tune/$v
  LD_LIBRARY_PATH=$lp timeout -k 10 120 python3 scripts/bench_physics.py --n 256 --steps 30 "$@" > $OUT/$v.$l.json 2> $OUT/$v.$l.err || { echo "$v $l rc=$?"; tail -3 $OUT/$v.$l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$v.$l.json'));print('$v','$l',d['ms_per_step'],d['last_path'])"
}
for rep in 1 2; do
  for v in base new new3 new3f; do
    run $v free; run $v nofree --no-free; run $v het --layers; run $v hetnofree --layers --no-free
  done
done
