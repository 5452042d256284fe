#!/bin/bash
# RCCL's split of the exchange group into kernel launches (N = 8 rank,
# 64x512x512 slab, one-rank self-exchange): for each RCCL setting, ms/step and
# RCCL kernels per step from a kernel trace.  Output under gpurun_out/r3/rcclenv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/rcclenv
mkdir -p $OUT
set -o pipefail
i=0
while read -r cfg; do
  [ -z "$cfg" ] && continue
  i=$((i+1))
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$i -o run -- \
    python3 scripts/bench_slab.py --ranks ${RANKS:-8} --steps 20 --reps 3 --rccl-self --no-check > $OUT/t$i.jsonl 2> $OUT/t$i.err \
    || { echo "cfg $i ($cfg) failed"; tail -5 $OUT/t$i.err; exit 1; }
  python3 - "$cfg" $OUT/t$i.jsonl $OUT/t$i/run_kernel_trace.csv <<'PY'
import csv, json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][0]
sys.argv[1] += f" ranks {d['ranks']}"
rows = list(csv.DictReader(open(sys.argv[3])))
nccl = [r for r in rows if "nccl" in r["Kernel_Name"].lower()]
steps = sum(1 for r in rows if "k_step_tx2" in r["Kernel_Name"]) / 2
print(f"{sys.argv[1]:60s} ms/step {d['ms_per_step']:.4f} reps {d['rep_ms_per_step']}  rccl kernels/step {len(nccl) / max(1, steps):.2f}")
PY
done < "${1:-scripts/rcclenv_cfgs.txt}"
