#!/bin/bash
# Round 5, lease I: the one-pass 2-D step (k_step2d): its parity tests, the
# parity / engine suites it now runs under, and its throughput against the two
# generic stages (scripts/bench_2d.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_2d.py tests/test_gpu_faces.py tests/test_gpu_parity.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $OUT/pytest.txt | head -20; exit $rc; }
timeout -k 10 300 python scripts/bench_2d.py > $OUT/bench_2d.jsonl 2> $OUT/bench_2d.err || { echo "bench_2d rc=$?"; tail -5 $OUT/bench_2d.err; exit 1; }
cat $OUT/bench_2d.jsonl
