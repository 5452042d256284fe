#!/bin/bash
# Round 5, lease Y: 256^3 across chunk sizes of the shuffled mapping on this
# box (hipMalloc, 16 / 32 / 64 / 128 / 256 / 512 MiB), then 512^3 default and
# hipMalloc for the box's context.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-y}
mkdir -p $OUT
b() {
  tag=$1; args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-copy-ceiling > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['process_state']['box'].get('unique_id'), d['process_state']['layers']['alloc'])" $OUT/b_$tag.json $tag
}
A="--n 256 --steps 100 --warmup 20 --reps 5"
for rep in 1 2; do
  for a in malloc shuffle:16 shuffle:32 shuffle:64 shuffle:128 shuffle:256 shuffle:512; do b ${a/:/}_256_$rep "$A" GCMX_ALLOC=$a; done
done
A="--steps 30 --warmup 5 --reps 5"
b def512 "$A" GCMX_NONE=1
b malloc512 "$A" GCMX_ALLOC=malloc
