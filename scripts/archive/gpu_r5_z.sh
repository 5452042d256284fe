#!/bin/bash
# Round 5, lease Z: prologue rows' loads one row ahead (tune/proahead) against
# the main build: the N = 8 slab's boundary launch (a 4-row march whose
# prologue is half its chain), 512^3 and 256^3, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-z}
mkdir -p $OUT
LP=gcm_amd/lib/tune/proahead/libgcmx.so
for rep in 1 2; do
  for v in main pro; do
    if [ $v = pro ]; then E="GCMX_LIB=$LP"; else E="GCMX_NONE=1"; fi
    env $E timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab_${v}_$rep.json 2> $OUT/slab_${v}_$rep.err || { echo "slab $v rc=$?"; exit 1; }
    python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);k=d['kernels']
print(sys.argv[2], 'slab8', d['ms_per_step'], 'boundary', k['fused_xyz_boundary'], 'interior', k['fused_xyz'])" $OUT/slab_${v}_$rep.json "$v$rep"
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b512_${v}_$rep.json 2> $OUT/b512_${v}_$rep.err || { echo "512 $v rc=$?"; exit 1; }
    env $E timeout -k 10 300 python bench.py --n 256 --steps 100 --warmup 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b256_${v}_$rep.json 2> $OUT/b256_${v}_$rep.err || { echo "256 $v rc=$?"; exit 1; }
    python3 -c "
import json,sys;a=json.load(open(sys.argv[1]));b=json.load(open(sys.argv[2]))
print(sys.argv[3], '512', a['roofline']['kernel_avg_ms'], '256', b['roofline']['kernel_avg_ms'], a['process_state']['box'].get('unique_id'))" $OUT/b512_${v}_$rep.json $OUT/b256_${v}_$rep.json "$v$rep"
  done
done
