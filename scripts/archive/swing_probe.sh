#!/bin/bash
# why the same build ran 4.22 ms/step bare and 3.92-4.02
# under rocprofv3 on one lease.  One lease, fresh processes back to back, every
# bench line carrying process_state (layer addresses and residues, the clock a
# co-resident wave sees, the allocation order).  Output: gpurun_out/r4/swing_$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/swing_${TAG:-a}
mkdir -p $OUT
BA="--steps 20 --warmup 5 --reps 5 --no-cpu-baseline"
summ() {
  python3 - "$1" <<'EOF'
import json, sys
f = sys.argv[1]
try:
    d = json.loads(open(f).read().strip().splitlines()[-1])
except Exception as e:
    print(f, "unreadable", e); sys.exit(0)
r = d.get("roofline") or {}
ps = d.get("process_state") or {}
L = ps.get("layers", {})
c = ps.get("clock") or {}
print(f"{f.split('/')[-1]:22s} step {d['ms_per_step']:.4f} kern {r.get('kernel_avg_ms')} frac {r.get('frac')} "
      f"copy {r.get('copy_ceiling', {}).get('GBps')} clk {c.get('mhz_median')} [{c.get('mhz_p10')},{c.get('mhz_p90')}] "
      f"a {L.get('a')} b-a {L.get('b_minus_a')} amod2M {L.get('a_mod', {}).get('2M')} one {L.get('one_allocation')}",
      flush=True)
EOF
}
run() {
  local name=$1; shift
  timeout -k 10 150 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; exit 1; }
  summ $OUT/$name.json
}
run bare1 python bench.py $BA
run bare2 python bench.py $BA
run noclock python bench.py $BA --no-clock-probe
run trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BA
run bare3 python bench.py $BA
run prio env GCMX_STREAM_PRIO=normal python bench.py $BA
for g in 1 2 4 8; do run pre$g python bench.py $BA --prealloc-gb $g; done
for gap in -1 0 4096 65536 2097152 1073741824; do run gap$gap env GCMX_LAYER_GAP=$gap python bench.py $BA; done
run emu8 python bench.py --emulate-slabs 8 --steps 5 --reps 2
run bare4 python bench.py $BA
run trace2 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace2 -o run -- python3 bench.py $BA
run bare5 python bench.py $BA
echo done
