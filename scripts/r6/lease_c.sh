#!/bin/bash
# Round 6, lease C: the z-split step (rows of 1024) -- parity tests, then the
# 1024^3 bench line; the padded-layout suite; the round-5 padded-build failure's
# hypothesis (two copies of libgcmx.so in one process: GCMX_LIB for ctypes, the
# rpath copy for the C++ engine), with and without the contiguous allocation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6/c
mkdir -p $OUT
PT="python -u -m pytest -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_parity.py -k "zsplit" tests/test_gpu_slabs.py -k "zsplit" > $OUT/pytest_zs.txt 2>&1
rc=$?; echo "zsplit tests rc=$rc"; grep -E "(PASSED|FAILED|ERROR)" $OUT/pytest_zs.txt | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 $PT tests/test_gpu_fma.py -k "1024" > $OUT/pytest_fma1024.txt 2>&1
echo "fma-1024 rc=$?"; tail -1 $OUT/pytest_fma1024.txt
timeout -k 10 300 $PT tests/test_gpu_layout.py > $OUT/pytest_layout.txt 2>&1
echo "layout rc=$?"; tail -1 $OUT/pytest_layout.txt
K="engine_two_layers or heterogeneous_within"
GCMX_ALLOC=contiguous timeout -k 10 200 $PT tests/test_gpu_fma.py -k "$K" > $OUT/hyp_one_copy_contig.txt 2>&1; echo "one copy, contiguous rc=$?"; tail -1 $OUT/hyp_one_copy_contig.txt
GCMX_LIB=gcm_amd/lib/tune/copy/libgcmx.so timeout -k 10 200 $PT tests/test_gpu_fma.py -k "$K" > $OUT/hyp_two_copies.txt 2>&1; echo "two copies rc=$?"; tail -1 $OUT/hyp_two_copies.txt
GCMX_LIB=gcm_amd/lib/tune/copy/libgcmx.so GCMX_ALLOC=contiguous timeout -k 10 200 $PT tests/test_gpu_fma.py -k "$K" > $OUT/hyp_two_copies_contig.txt 2>&1; echo "two copies, contiguous rc=$?"; tail -1 $OUT/hyp_two_copies_contig.txt
timeout -k 10 500 python bench.py --n 1024 --steps 5 --warmup 2 --reps 3 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_1024.json 2> $OUT/bench_1024.err || { echo "bench 1024 rc=$?"; tail -5 $OUT/bench_1024.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_1024.json'));r=d['roofline'];print('1024',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel_symbol'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_512.json 2> $OUT/bench_512.err || { echo "bench 512 rc=$?"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_512.json'));r=d['roofline'];print('512',d['ms_per_step'],r['kernel_avg_ms'],r['frac'],r['kernel_symbol'])"
