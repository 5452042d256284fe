#!/bin/bash
# Tuning only: time the simplex 16^3 cube step with diagnostic builds of libgcmx.so
# (gcm_amd/lib/sxtune/NAME) swapped in place on the GPU box's copy of the tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sxv
mkdir -p gcm_amd/lib/sxtune && cp gcm_amd/lib/libgcmx.so gcm_amd/lib/sxtune/base.so
for d in base $(ls -d gcm_amd/lib/sxtune/*/ 2>/dev/null); do
  name=$(basename "$d")
  if [ "$name" = base ]; then cp gcm_amd/lib/sxtune/base.so gcm_amd/lib/libgcmx.so; else cp "$d/libgcmx.so" gcm_amd/lib/libgcmx.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sxv/$name -o run -- \
    python3 scripts/bench_simplex.py --n 16 --steps 20 --warmup 3 --workloads cube --lanes 8 > gpurun_out/sxv/$name.json 2> gpurun_out/sxv/$name.err || exit 1
  python3 - gpurun_out/sxv/$name/run_kernel_stats.csv $name <<'PY'
import csv, sys
print(sys.argv[2], "  ".join(f"{r['Name'].split('(')[1].split('::')[-1] if '::' in r['Name'] else r['Name'][:20]} {float(r['AverageNs'])/1000:.2f}" for r in csv.DictReader(open(sys.argv[1])) if 'k_sx' in r['Name']))
PY
done
cp gcm_amd/lib/sxtune/base.so gcm_amd/lib/libgcmx.so
