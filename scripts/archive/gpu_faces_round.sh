cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/faces
timeout -k 10 600 python -u -m pytest tests/test_gpu_faces.py -v -x --timeout 300 --timeout-method thread > gpurun_out/faces/pytest_faces.log 2>&1
rc=$?; tail -20 gpurun_out/faces/pytest_faces.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/faces/pytest_all.log 2>&1
rc=$?; tail -5 gpurun_out/faces/pytest_all.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_physics.py --n 512 --steps 10 > gpurun_out/faces/phys512.json 2> gpurun_out/faces/phys512.err
rc=$?; cat gpurun_out/faces/phys512.json; tail -2 gpurun_out/faces/phys512.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --n 512 --reps 3 --no-cpu-baseline > gpurun_out/faces/bench512.json 2> gpurun_out/faces/bench512.err
rc=$?; cat gpurun_out/faces/bench512.json; [ $rc -eq 0 ] || exit $rc
