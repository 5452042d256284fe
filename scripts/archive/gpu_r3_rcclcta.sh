#!/bin/bash
# One N = 8 rank (64x512x512 slab) with the real RCCL self-exchange in flight:
# the communicator's CTA request swept (GCMX_COMM_MIN_CTAS / MAX_CTAS; 0 = RCCL's
# own choice), then a kernel trace of the default.  Output under gpurun_out/r3/rcclcta.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/rcclcta
mkdir -p $OUT
set -o pipefail
for cfg in "0 0" "4 8" "8 16" "16 32" "32 64"; do
  set -- $cfg
  GCMX_COMM_MIN_CTAS=$1 GCMX_COMM_MAX_CTAS=$2 timeout -k 10 120 python scripts/bench_slab.py --ranks 8 --steps 30 --rccl-self --no-check \
    > $OUT/cta_$1_$2.jsonl 2> $OUT/cta.err || { tail $OUT/cta.err; exit 1; }
  echo "min $1 max $2: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(d['ms_per_step'], d['rep_ms_per_step'])" $OUT/cta_$1_$2.jsonl)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 scripts/bench_slab.py --ranks 8 --steps 30 --reps 2 --rccl-self --no-check > $OUT/trace.jsonl 2> $OUT/trace.err \
  || { tail $OUT/trace.err; exit 1; }
python scripts/trace_gaps.py $OUT/trace/run_kernel_trace.csv 40
python scripts/trace_timeline.py $OUT/trace/run_kernel_trace.csv 60 16
