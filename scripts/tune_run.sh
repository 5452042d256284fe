#!/bin/bash
# On the GPU box: bench every variant in gcm_amd/lib/tune/ (512^3, fused path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tune
for d in gcm_amd/lib/tune/*/; do
  n=$(basename $d)
  GCMX_LIB=$d/libgcmx.so timeout -k 10 120 python3 bench.py --n ${N:-512} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
    > gpurun_out/tune/$n.json 2> gpurun_out/tune/$n.err
  rc=$?
  echo "$n rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/tune/$n.json')); print(d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['roofline']['kernels'].items()})" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
