#!/bin/bash
# N = 4 and N = 8 ranks with the one-rank RCCL self-exchange: RCCL's default
# channels per peer against the library's 8, each in its own process, with a
# kernel trace.  Output under gpurun_out/r3/rccl4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/rccl4
mkdir -p $OUT
set -o pipefail
for r in 4 8; do
for ch in 0 8 4; do
  GCMX_COMM_CHANNELS_PER_PEER=$ch timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/r${r}_c$ch -o run -- \
    python3 scripts/bench_slab.py --ranks $r --steps 20 --reps 3 --rccl-self --no-check > $OUT/r${r}_c$ch.jsonl 2> $OUT/r${r}_c$ch.err \
    || { tail -5 $OUT/r${r}_c$ch.err; exit 1; }
  python3 - $r $ch $OUT/r${r}_c$ch.jsonl $OUT/r${r}_c$ch/run_kernel_trace.csv <<'PY'
import csv, json, sys, statistics
d = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")][0]
rows = sorted(csv.DictReader(open(sys.argv[4])), key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if "k_step" in r["Kernel_Name"] or "nccl" in r["Kernel_Name"].lower()]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
ks = [r for r in sel if "k_step" in r["Kernel_Name"]]
gx = sorted({r["Grid_Size_X"] for r in ks})
by = {g: statistics.median([dur(r) for r in ks if r["Grid_Size_X"] == g]) for g in gx}
nc = [dur(r) for r in sel if "nccl" in r["Kernel_Name"].lower()]
print(f"ranks {sys.argv[1]} channels {sys.argv[2]}: ms/step {d['ms_per_step']} reps {d['rep_ms_per_step']} "
      f"step kernels by grid {by} rccl per step {len(nc) / (len(ks) / 2):.2f} median {statistics.median(nc):.1f} us")
n = len(sel)
sl = sel[n // 2:n // 2 + 8]
t0 = int(sl[0]["Start_Timestamp"])
for r in sl:
    print(f"   {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f} {dur(r):8.1f} "
          f"{'nccl' if 'nccl' in r['Kernel_Name'].lower() else 'step'} grid={r['Grid_Size_X']}")
PY
done
done
