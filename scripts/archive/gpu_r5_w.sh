#!/bin/bash
# Round 5, lease W: the copy ceiling with the layers' placement (shuffled chunks)
# against hipMalloc buffers, beside the step; the slab / measurement suites.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-w}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_measure.py tests/test_gpu_slabs.py tests/test_gpu_biggrid.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for a in default malloc; do
    if [ $a = malloc ]; then E="GCMX_ALLOC=malloc"; else E="GCMX_NONE=1"; fi
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --reps 5 --no-cpu-baseline > $OUT/b_${a}_$rep.json 2> $OUT/b_${a}_$rep.err || { echo "$a rc=$?"; exit 1; }
    python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];c=r['copy_ceiling']
print(sys.argv[2], d['ms_per_step'], r['kernel_avg_ms'], r['frac'], 'copy', c['GBps'], c['frac_of_copy'], d['process_state']['box'].get('unique_id'), d['process_state']['layers']['alloc'])" $OUT/b_${a}_$rep.json "$a$rep"
  done
done
