#!/bin/bash
# Time every variant under gcm_amd/lib/tune on one box (same GPU, back to back):
# one bench.py line each, then a summary.  N (default 512), STEPS (20).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
for d in gcm_amd/lib/tune/*/; do
  name=$(basename "$d")
  if [ $rep = 1 ]; then
    GCMX_FP=exact GCMX_LIB="$d/libgcmx.so" timeout -k 10 120 python scripts/ab_check.py > gpurun_out/ab/$name.check 2>&1
    rc=$?; echo "$name: $(tail -1 gpurun_out/ab/$name.check)"
    [ $rc -le 1 ] || exit $rc
  fi
  GCMX_LIB="$d/libgcmx.so" timeout -k 10 300 python bench.py --n ${N:-512} --steps ${STEPS:-20} \
    --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/$name.$rep.json 2> gpurun_out/ab/$name.$rep.err
  rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 gpurun_out/ab/$name.$rep.err; exit $rc; }
  python - "$name" gpurun_out/ab/$name.$rep.json <<'PY'
import json, sys
r = json.load(open(sys.argv[2]))
ks = r["roofline"]["kernels"] if r.get("roofline") else {}
print(f"{sys.argv[1]:>14s} {r['value']:9.1f} Mnode-steps/s  " +
      "  ".join(f"{k} {v['avg_ms']:.3f}ms" for k, v in ks.items()))
PY
done
done
