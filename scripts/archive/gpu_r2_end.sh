#!/bin/bash
# Round-2 end check on one MI355X: the whole -m gpu suite, smoke, the default
# bench line (copy ceiling included), the 256^3 config, the hot kernel's
# rocprofv3 kernel trace and FETCH/WRITE passes (gpu_profile.sh).  Output under
# gpurun_out/r2end/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2end
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_512.json 2> $O/bench_512.err || { tail $O/bench_512.err; exit 1; }
cat $O/bench_512.json
timeout -k 10 300 python bench.py --n 256 --no-cpu-baseline > $O/bench_256.json 2> $O/bench_256.err || exit 1
TAG=r2end bash scripts/gpu_profile.sh > $O/profile.log 2>&1 || { tail $O/profile.log; exit 1; }
tail -3 $O/profile.log
