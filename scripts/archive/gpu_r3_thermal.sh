#!/bin/bash
# Does the 512^3 step slow down after sustained load (the GPU test suite)?
# bench right after the suite, after 60 s idle, and a 200-step run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3/thermal; mkdir -p $OUT
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-copy-ceiling "$@" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['rep_ms_per_step'])"; }
echo "cold: $(b)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -5 $OUT/pytest.txt; exit 1; }
echo "after suite: $(b)"
sleep 60
echo "after 60 s idle: $(b)"
echo "200 steps x 3 reps: $(b --steps 200 --reps 3)"
