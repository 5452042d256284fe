#!/bin/bash
# Simplex kernel roofline inputs: rocprofv3 kernel stats of the 64^3 cube in the
# throughput layout (one thread per node) and of the 16^3 cube (eight lanes,
# one-launch stage).  Output under gpurun_out/sxr/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sxr
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sxr/n64 -o run -- \
  python3 scripts/bench_simplex.py --n 64 --steps 20 --warmup 2 --workloads cube --lanes 1 > gpurun_out/sxr/n64.json 2> gpurun_out/sxr/n64.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sxr/n16 -o run -- \
  python3 scripts/bench_simplex.py --n 16 --steps 200 --warmup 5 --workloads cube > gpurun_out/sxr/n16.json 2> gpurun_out/sxr/n16.err || exit 1
for f in n64 n16; do
python3 - gpurun_out/sxr/$f/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_sx' in r['Name']:
        print(r['Name'].split('(')[1].split('::')[-1] if '::' in r['Name'] else r['Name'][:30], r['Calls'], round(float(r['AverageNs']) / 1000, 2), 'us')
PY
done
cat gpurun_out/sxr/n64.json gpurun_out/sxr/n16.json
