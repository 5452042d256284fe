#!/bin/bash
# Round 4, lease e: A/B of the FACES / HET costs at 256^3 (bench_physics wall
# time per step; variants from scripts/ab_build.sh, loaded through
# LD_LIBRARY_PATH ahead of the engine's RUNPATH).  Output under gpurun_out/r4/e.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/e
mkdir -p $OUT
run() {  # variant, label, args...
  local v=$1 l=$2; shift 2
  local lp=""
  [ "$v" = base ] || lp=gcm_amd/lib/tune/$v
  LD_LIBRARY_PATH=$lp timeout -k 10 120 python3 scripts/bench_physics.py --n 256 --steps 30 "$@" > $OUT/$v.$l.json 2> $OUT/$v.$l.err || { echo "$v $l rc=$?"; tail -3 $OUT/$v.$l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$v.$l.json'));print('$v','$l',d['ms_per_step'],d['last_path'])"
}
for rep in 1 2; do
  for v in base nomap flds lastrow new; do run $v free; done
  for v in base lastrow new; do run $v nofree --no-free; done
  for v in base hettab hetnoid lastrow new; do run $v het --layers; run $v hetnofree --layers --no-free; done
done
