#!/bin/bash
# Round 4: chunk-minor vs chunk-major block order (A/B at 256^3 and the 8-slab emulation).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4/cminor; mkdir -p $OUT gpurun_out/ab
N=256 bash scripts/ab_run.sh > $OUT/ab256.txt 2>&1 || exit 1
cat $OUT/ab256.txt
for rep in 1 2; do for v in base cminor; do
  GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so timeout -k 10 200 python bench.py --emulate-slabs 8 --steps 10 --reps 3 > $OUT/emu8_${v}_$rep.json 2> $OUT/emu8_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/emu8_${v}_$rep.json'));print('emu8 $v',d['ms_per_step'])"
done; done
