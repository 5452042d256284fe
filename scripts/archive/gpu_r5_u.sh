#!/bin/bash
# Round 5, lease U: chunk size of the shuffled mapping for the smaller blocks
# (256^3, the N = 8 slab, 2-D 8192^2): hipMalloc, 64 MiB and 256 MiB chunks,
# two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-u}
mkdir -p $OUT
for rep in 1 2; do
  for a in malloc shuffle:64 shuffle:256; do
    t=${a/:/}_$rep
    GCMX_ALLOC=$a timeout -k 10 300 python bench.py --n 256 --steps 100 --warmup 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b256_$t.json 2> $OUT/b256_$t.err || { echo "256 $a rc=$?"; exit 1; }
    GCMX_ALLOC=$a timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8_$t.json 2> $OUT/slab8_$t.err || { echo "slab $a rc=$?"; exit 1; }
    GCMX_ALLOC=$a timeout -k 10 300 python scripts/bench_2d.py --steps 50 > $OUT/b2d_$t.jsonl 2> $OUT/b2d_$t.err || { echo "2d $a rc=$?"; exit 1; }
    python3 - $OUT $t <<'PY'
import json, sys
out, t = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/b256_{t}.json"))
s = json.loads(open(f"{out}/slab8_{t}.json").read().strip().splitlines()[-1])
two = [json.loads(l) for l in open(f"{out}/b2d_{t}.jsonl") if "8192" in l and '"fused"' in l][0]
print(t, "256:", d["roofline"]["kernel_avg_ms"], "slab8:", s["ms_per_step"], "2d:", two["kernels"]["step2d"]["avg_ms"], d["process_state"]["box"].get("unique_id"))
PY
  done
done
