#!/bin/bash
# Tuning only: the one-launch simplex stage's wait modes (GCMX_SX_WAIT_MODE builds
# under gcm_amd/lib/sxtune/NAME) swapped in place, each checked against the
# two-launch stage bitwise and timed per kernel at 16^3 (fused and split).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sxw
cp gcm_amd/lib/libgcmx.so gcm_amd/lib/sxtune/base.so
for name in base w0 w2 base; do
  if [ "$name" = base ]; then cp gcm_amd/lib/sxtune/base.so gcm_amd/lib/libgcmx.so; else cp gcm_amd/lib/sxtune/$name/libgcmx.so gcm_amd/lib/libgcmx.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_simplex.py -q -x -k one_launch --timeout 120 --timeout-method thread > gpurun_out/sxw/$name.pytest 2>&1 || { tail -5 gpurun_out/sxw/$name.pytest; exit 1; }
  for f in "" "--no-fusion"; do
    tag=$name$f
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sxw/$tag -o run -- \
      python3 scripts/bench_simplex.py --n 16 --steps 200 --warmup 5 --workloads cube,fracture $f > gpurun_out/sxw/$tag.json 2> gpurun_out/sxw/$tag.err || exit 1
    python3 - gpurun_out/sxw/$tag/run_kernel_stats.csv $tag gpurun_out/sxw/$tag.json <<'PY'
import csv, sys, json
ms = [json.loads(l)["ms_per_step"] for l in open(sys.argv[3])]
print(f"{sys.argv[2]:18s} step(cube,frac) {ms}", "  ".join(f"{r['Name'].split('(')[1].split('::')[-1] if '::' in r['Name'] else r['Name'][:20]} {float(r['AverageNs'])/1000:.2f}" for r in csv.DictReader(open(sys.argv[1])) if 'k_sx' in r['Name']))
PY
  done
done
cp gcm_amd/lib/sxtune/base.so gcm_amd/lib/libgcmx.so
