#!/bin/bash
# Round 5, lease N: is the 512^3 step's per-device spread a translation (TLB)
# effect?  UTCL1 translation hits / misses per launch of the step at 512^3 and
# 256^3 (256^3 runs equally fast on the slow devices), with the layers from
# hipMalloc and from a physically contiguous allocation (tune/contig,
# GCMX_ALLOC=contiguous), then the bench A/B of the two allocations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-n}
mkdir -p $OUT
bash scripts/box_char.sh $OUT > $OUT/box_char.log 2>&1 || { echo "box_char failed"; tail -5 $OUT/box_char.log; exit 1; }
tail -1 $OUT/box_char.log
CT="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum"
BP="--steps 3 --warmup 1 --reps 1 --no-cpu-baseline --no-profile --no-copy-ceiling --no-clock-probe --no-box-state"
timeout -k 10 150 rocprofv3 --pmc $CT --output-format csv -d $OUT/tlb512 -o run -- python3 bench.py --n 512 $BP > $OUT/tlb512.json 2> $OUT/tlb512.err || { echo "tlb512 rc=$?"; tail -3 $OUT/tlb512.err; exit 1; }
echo "tlb512 ok"
timeout -k 10 150 rocprofv3 --pmc $CT --output-format csv -d $OUT/tlb256 -o run -- python3 bench.py --n 256 $BP > $OUT/tlb256.json 2> $OUT/tlb256.err || { echo "tlb256 rc=$?"; tail -3 $OUT/tlb256.err; exit 1; }
echo "tlb256 ok"
GCMX_LIB=gcm_amd/lib/tune/contig/libgcmx.so GCMX_ALLOC=contiguous timeout -k 10 150 rocprofv3 --pmc $CT --output-format csv -d $OUT/tlb512c -o run -- python3 bench.py --n 512 $BP > $OUT/tlb512c.json 2> $OUT/tlb512c.err || { echo "tlb512c rc=$?"; tail -3 $OUT/tlb512c.err; exit 1; }
echo "tlb512c ok"; grep -i contiguous $OUT/tlb512c.err | head -2
BA="--steps 50 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
for rep in 1 2; do
  for v in def contig; do
    if [ $v = contig ]; then
      GCMX_LIB=gcm_amd/lib/tune/contig/libgcmx.so GCMX_ALLOC=contiguous timeout -k 10 200 python bench.py $BA > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { echo "$v rc=$?"; exit 1; }
    else
      timeout -k 10 200 python bench.py $BA > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { echo "$v rc=$?"; exit 1; }
    fi
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'],d['process_state']['env'])" $OUT/ab_${v}_$rep.json "$v rep$rep"
  done
done
grep -i contiguous $OUT/ab_contig_1.err | head -2
