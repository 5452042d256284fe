#!/bin/bash
# Round 5, lease V: with the shuffled placement, re-measure choices made under
# hipMalloc placement: rows per block at 256^3 / 512^3 (runtime), non-temporal
# outermost-plane loads (tune/ntouter) and plain stores (tune/stnt0), A/B
# alternating against the main build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-v}
mkdir -p $OUT
b() {
  tag=$1; args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-copy-ceiling > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['process_state']['box'].get('unique_id'), d['process_state']['layers']['alloc'])" $OUT/b_$tag.json $tag
}
A512="--steps 30 --warmup 5 --reps 5"
for rep in 1 2; do
  b main512_$rep "$A512" GCMX_NONE=1
  b ntouter512_$rep "$A512" GCMX_LIB=gcm_amd/lib/tune/ntouter/libgcmx.so
  b stnt0_512_$rep "$A512" GCMX_LIB=gcm_amd/lib/tune/stnt0/libgcmx.so
  b rows256_512_$rep "$A512 --rows-per-block 256" GCMX_NONE=1
done
A256="--n 256 --steps 100 --warmup 20 --reps 5"
for rep in 1 2; do
  for r in 64 32 128; do b r${r}_256_$rep "$A256 --rows-per-block $r" GCMX_NONE=1; done
  b ntouter256_$rep "$A256" GCMX_LIB=gcm_amd/lib/tune/ntouter/libgcmx.so
done
