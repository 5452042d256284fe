#!/bin/bash
# Round 5, lease K: where the N = 8 slab step's time goes.  rocprofv3 kernel
# trace of the 64 x 512^2 slab with the real RCCL self-exchange (per-dispatch
# timeline: boundary launch, RCCL kernel, interior), then the boundary rows per
# block (GCMX_BOUNDARY_ROWS) swept without and with the exchange.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-k}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_slab8 -o slab8 -- python3 scripts/bench_slab.py --rccl-self --ranks 8 --no-check --steps 20 --reps 3 > $OUT/prof_slab8.json 2> $OUT/prof_slab8.err || { echo "prof rc=$?"; tail -5 $OUT/prof_slab8.err; exit 1; }
cat $OUT/prof_slab8.json
for br in 2 4 8; do
  GCMX_BOUNDARY_ROWS=$br timeout -k 10 200 python scripts/bench_slab.py --ranks 8 --no-check > $OUT/slab8_br$br.json 2> $OUT/slab8_br$br.err || { echo "br$br rc=$?"; tail -3 $OUT/slab8_br$br.err; exit 1; }
  echo "br=$br noex"; python3 -c "import json,sys;d=[json.loads(l) for l in open(sys.argv[1])][-1];print(d['ms_per_step'], d.get('kernels'))" $OUT/slab8_br$br.json
  GCMX_BOUNDARY_ROWS=$br timeout -k 10 200 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8r_br$br.json 2> $OUT/slab8r_br$br.err || { echo "br$br rccl rc=$?"; tail -3 $OUT/slab8r_br$br.err; exit 1; }
  echo "br=$br rccl"; python3 -c "import json,sys;d=[json.loads(l) for l in open(sys.argv[1])][-1];print(d['ms_per_step'], d.get('kernels'))" $OUT/slab8r_br$br.json
done
