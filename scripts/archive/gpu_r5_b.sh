#!/bin/bash
# Round 5, lease B: the z-grouping access-pattern probe (two planes x two z
# groups per lane at one wave per SIMD), a long 512^3 bench
# for steady power / clock readings, the slab / RCCL tests of the new build
# (checked channels contract, exchange timings), and a one-rank RCCL
# self-exchange bench line with per_rank (item 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-b}
mkdir -p $OUT
TZ_ONLY=1 PROBE_REPS=300 timeout -k 10 240 python3 tools/power_probe.py $OUT/xyz_probe_tz.json -- ./tools/xyz_probe > $OUT/xyz_probe_tz.txt 2>&1; rc=$?; echo "probe rc=$rc"; cat $OUT/xyz_probe_tz.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_slabs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_slabs.txt 2>&1
rc=$?; echo "pytest slabs rc=$rc"; tail -3 $OUT/pytest_slabs.txt
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];b=d['process_state'].get('box_during_reps') or {}
print(sys.argv[2],d['ms_per_step'],r['kernel_avg_ms'],r['frac'],'power',b.get('power_w'),'sclk',b.get('sclk'))" "$1" "$2"; }
timeout -k 10 300 python bench.py --steps 100 --reps 7 --no-cpu-baseline > $OUT/bench_long.json 2> $OUT/bench_long.err || { echo "bench rc=$?"; tail -5 $OUT/bench_long.err; exit 1; }
summ $OUT/bench_long.json long512
timeout -k 10 300 python bench.py --rccl-self --steps 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/bench_rccl_self.json 2> $OUT/bench_rccl_self.err || { echo "rccl-self rc=$?"; tail -5 $OUT/bench_rccl_self.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_rccl_self.json'));print('rccl-self', d['ms_per_step'], d['per_rank'])"
timeout -k 10 300 python scripts/bench_slab.py --rccl-self --ranks 8 --no-check > $OUT/slab8_rccl_self.json 2> $OUT/slab8_rccl_self.err || { echo "slab8 rc=$?"; tail -5 $OUT/slab8_rccl_self.err; exit 1; }
tail -1 $OUT/slab8_rccl_self.json
