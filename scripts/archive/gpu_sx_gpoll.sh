#!/bin/bash
# Tuning only: gradient-counter poll interval of the mode-2 one-launch stage
# (GCMX_SX_GPOLL_SLEEP builds under gcm_amd/lib/sxtune/gpN), 16^3 cube/fracture.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gp && rm -f gpurun_out/gp/b.jsonl
cp gcm_amd/lib/libgcmx.so gcm_amd/lib/sxtune/base.so
for name in base gp8 gp32 gp127; do
  if [ "$name" = base ]; then cp gcm_amd/lib/sxtune/base.so gcm_amd/lib/libgcmx.so; else cp gcm_amd/lib/sxtune/$name/libgcmx.so gcm_amd/lib/libgcmx.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_simplex.py -q -x -k "one_launch and gradient" --timeout 120 --timeout-method thread > gpurun_out/gp/$name.pytest 2>&1 || { tail -5 gpurun_out/gp/$name.pytest; exit 1; }
  for f in 2 1; do
    echo "{\"build\": \"$name\"}" >> gpurun_out/gp/b.jsonl
    timeout -k 10 200 python scripts/bench_simplex.py --n 16 --steps 400 --warmup 10 --workloads cube,fracture --fusion $f >> gpurun_out/gp/b.jsonl || exit 1
  done
done
cp gcm_amd/lib/sxtune/base.so gcm_amd/lib/libgcmx.so
python3 -c "
import json
b = ''
for l in open('gpurun_out/gp/b.jsonl'):
    r = json.loads(l)
    if 'build' in r: b = r['build']; continue
    print(b, r['workload'], 'fusion', r['fusion'], r['ms_per_step'])"
