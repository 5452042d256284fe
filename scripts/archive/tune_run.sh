#!/bin/bash
# On the GPU box: parity-check then bench every variant in gcm_amd/lib/tune/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tune
for d in gcm_amd/lib/tune/*/; do
  n=$(basename $d)
  GCMX_LIB=$d/libgcmx.so timeout -k 10 300 python3 -m pytest -q -m gpu tests/test_gpu_parity.py -k "fused or split or anchor or slabs" \
    > gpurun_out/tune/$n.pytest 2>&1
  prc=$?
  [ $prc -le 1 ] || { echo "$n pytest rc=$prc"; exit $prc; }
  GCMX_LIB=$d/libgcmx.so timeout -k 10 120 python3 bench.py --n ${N:-512} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
    > gpurun_out/tune/$n.json 2> gpurun_out/tune/$n.err
  rc=$?
  echo "$n parity=$(tail -1 gpurun_out/tune/$n.pytest) rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/tune/$n.json')); print(d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['roofline']['kernels'].items()})" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
