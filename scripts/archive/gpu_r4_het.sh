#!/bin/bash
# Round 4: the heterogeneous record for the last build -- 256^3 two materials
# with free surfaces (and + Maxwell), wall time and rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4/het_final
mkdir -p $OUT
for a in "het:--layers" "hetmax:--layers --maxwell" "free:" "nofree:--no-free"; do
  n=${a%%:*}; args=${a#*:}
  timeout -k 10 200 python3 scripts/bench_physics.py --n 256 --steps 50 $args > $OUT/$n.json 2> $OUT/$n.err || { echo "$n rc=$?"; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$n -o run -- python3 scripts/bench_physics.py --n 256 --steps 50 $args > $OUT/${n}_traced.json 2> $OUT/${n}_traced.err || { echo "$n trace rc=$?"; exit 1; }
  python3 - $OUT $n <<'PY'
import csv, glob, json, sys
out, n = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/{n}.json"))
rows = list(csv.DictReader(open(glob.glob(f"{out}/trace_{n}/**/*kernel_stats.csv", recursive=True)[0])))
k = [r for r in rows if "k_step_tx2" in r["Name"]][0]
print(f"{n:7s} wall {d['ms_per_step']:.4f} ms/step  kernel avg {float(k['AverageNs'])/1e6:.4f} ms  {k['Name'][:80]}")
PY
done
