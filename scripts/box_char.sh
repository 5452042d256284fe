#!/bin/bash
# Box characterisation, run at the start of a lease:
# the flat HBM copy and an fp64-FMA-only kernel, each alone, with the power
# and sclk sampled from sysfs (tools/power_probe.py), then a steady 512^3 bench
# (100 steps x 7) whose line carries the box's sysfs state.  Usage:
#   bash scripts/box_char.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r5/box}
mkdir -p $OUT
BOX_ONLY=1 PROBE_REPS=150 timeout -k 10 120 python3 tools/power_probe.py $OUT/box_probe.json -- ./tools/xyz_probe > $OUT/box_probe.txt 2>&1 || { echo "box probe rc=$?"; cat $OUT/box_probe.txt; exit 1; }
cat $OUT/box_probe.txt
timeout -k 10 300 python bench.py --steps 100 --reps 7 --no-cpu-baseline > $OUT/bench_long.json 2> $OUT/bench_long.err || { echo "bench rc=$?"; tail -5 $OUT/bench_long.err; exit 1; }
python3 - $OUT/bench_long.json <<'PY'
import json, statistics, sys
d = json.load(open(sys.argv[1])); ps = d["process_state"]; b = ps["box"]; s = ps["box_during_reps"] or {}
sc = [int(k[:-3]) for k, n in (s.get("sclk") or {}).items() for _ in range(n)]
print("box", b.get("unique_id"), b.get("vbios_version"), "smc", (b.get("fw_version") or {}).get("smc_fw_version"),
      "| 512^3 kernel", d["roofline"]["kernel_avg_ms"], "frac", d["roofline"]["frac"],
      "copy", (d["roofline"].get("copy_ceiling") or {}).get("GBps"), "power", s.get("power_w"),
      "sclk med", statistics.median(sc) if sc else None, "temps", s.get("temps_c_max"))
PY
