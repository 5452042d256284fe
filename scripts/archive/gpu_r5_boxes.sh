#!/bin/bash
# Round 5: one more box's sample of the shipped build -- 512^3 with the default
# (shuffled) placement and with hipMalloc, 256^3 default.  LEASE names the run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-boxes}
mkdir -p $OUT
b() {
  tag=$1; args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-copy-ceiling > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { echo "bench $tag rc=$?"; tail -3 $OUT/b_$tag.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['process_state']['box'].get('unique_id'), d['process_state']['box'].get('vbios_version'), d['process_state']['layers']['alloc'])" $OUT/b_$tag.json $tag
}
b def512 "--steps 20 --warmup 3 --reps 7" GCMX_NONE=1
b malloc512 "--steps 20 --warmup 3 --reps 7" GCMX_ALLOC=malloc
b def256 "--n 256 --steps 100 --warmup 20 --reps 5" GCMX_NONE=1
