#!/bin/bash
# Round 6: the final build's default bench line and the 256^3 line on whatever
# box this lease gets (box-to-box spread of the final build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/boxes/${1:-x}
mkdir -p $OUT
timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_512.json 2> $OUT/bench_512.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 200 python bench.py --n 256 --steps 100 --warmup 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_256.json 2> $OUT/bench_256.err || { echo "bench256 rc=$?"; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
d = json.load(open(f"{o}/bench_512.json")); r = d["roofline"]
e = json.load(open(f"{o}/bench_256.json")); q = e["roofline"]
print("box", d["process_state"]["box"].get("unique_id"), "| 512:", d["ms_per_step"], r["kernel_avg_ms"], r["frac"],
      "copy", r["copy_ceiling"]["frac_of_copy"], "traffic", r["traffic"] is not None, "| 256:", q["kernel_avg_ms"], q["frac"])
PY
