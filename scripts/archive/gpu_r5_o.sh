#!/bin/bash
# Round 5, lease O: does counter collection leave the GPU slow?  The same
# 512^3 bench before and after one rocprofv3 --pmc run of a small program,
# then after an idle minute and after a --kernel-trace-only run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-o}
mkdir -p $OUT
BA="--steps 30 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling"
b() {
  timeout -k 10 200 python bench.py $BA > $OUT/b_$1.json 2> $OUT/b_$1.err || { echo "bench $1 rc=$?"; exit 1; }
  python3 -c "
import json,statistics,sys;d=json.load(open(sys.argv[1]));s=d['process_state'].get('box_during_reps') or {}
sc=[int(k[:-3]) for k,n in (s.get('sclk') or {}).items() for _ in range(n)]
print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], 'power', (s.get('power_w') or {}).get('median'), 'sclk', statistics.median(sc) if sc else None, d['process_state']['box'].get('unique_id'))" $OUT/b_$1.json $1
}
b 1_start
b 2_again
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py --n 64 --steps 3 --warmup 1 --reps 1 --no-cpu-baseline --no-profile --no-copy-ceiling --no-clock-probe > $OUT/pmc1.json 2> $OUT/pmc1.err || { echo "pmc rc=$?"; exit 1; }
echo "pmc run done"
b 3_after_pmc
b 4_after_pmc
sleep 60
b 5_after_idle
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 bench.py --n 64 --steps 3 --warmup 1 --reps 1 --no-cpu-baseline --no-copy-ceiling --no-clock-probe > $OUT/kt.json 2> $OUT/kt.err || { echo "kt rc=$?"; exit 1; }
b 6_after_ktrace
