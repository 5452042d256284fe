#!/bin/bash
# Round 5, lease J: 2-D step A/B over library variants, alternating:
# VARIANTS (default "nt1 nt0": non-temporal stores against plain), each
# gcm_amd/lib/tune/<v>/libgcmx.so, "cur" = gcm_amd/lib/libgcmx.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-j}
mkdir -p $OUT
for rep in 1 2; do
  for v in ${VARIANTS:-cur pf2 pf3}; do
    if [ $v = cur ]; then L=gcm_amd/lib/libgcmx.so; else L=gcm_amd/lib/tune/$v/libgcmx.so; fi
    GCMX_LIB=$L timeout -k 10 200 python scripts/bench_2d.py --steps 100 > $OUT/b2d_${v}_$rep.jsonl 2> $OUT/b2d_${v}_$rep.err || { echo "$v rc=$?"; tail -3 $OUT/b2d_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys;[print(sys.argv[1], d['workload'], d['path'], d['ms_per_step'], [(k, v['avg_ms'], v['frac']) for k, v in d['kernels'].items()]) for d in map(json.loads, open(sys.argv[2]))]" "$v rep$rep" $OUT/b2d_${v}_$rep.jsonl
  done
done
