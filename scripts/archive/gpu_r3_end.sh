#!/bin/bash
# Round-3 check of the whole tree on one MI355X: the -m gpu suite in one
# process, smoke, the default bench line, 256^3, the X-slab group emulation
# (boundary-first schedule with the in-process exchange), the simplex config-4
# task and 16^3 cube, then the hot kernel's rocprofv3 kernel trace and
# FETCH/WRITE passes (gpu_profile.sh).  Output under gpurun_out/r3/$TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-end}
mkdir -p $OUT
set -o pipefail
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.txt
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python bench.py > $OUT/bench_512.json 2> $OUT/bench_512.err || { tail $OUT/bench_512.err; exit 1; }
cat $OUT/bench_512.json
timeout -k 10 300 python bench.py --n 256 --steps 50 --no-cpu-baseline > $OUT/bench_256.json 2> $OUT/bench_256.err || exit 1
for K in ${SLABS:-8 4 2}; do
  timeout -k 10 300 python bench.py --emulate-slabs $K --steps 10 --reps 5 > $OUT/emulate_$K.json 2> $OUT/emulate_$K.err \
    || { echo "emulate $K rc=$?"; tail $OUT/emulate_$K.err; exit 1; }
done
timeout -k 10 200 python scripts/bench_slab.py --ranks 8,4,2 --steps 30 > $OUT/slab.jsonl 2> $OUT/slab.err || { tail $OUT/slab.err; exit 1; }
timeout -k 10 200 python scripts/bench_slab.py --ranks 8,4,2 --steps 30 --loop-gbps 64 --no-check > $OUT/slab_loop64.jsonl 2>> $OUT/slab.err || { tail $OUT/slab.err; exit 1; }
: > $OUT/slab_rccl_self.jsonl
for r in 8 4 2; do  # one process per slab size: the first communicator fixes RCCL's channels per peer
  timeout -k 10 200 python scripts/bench_slab.py --ranks $r --steps 30 --rccl-self --no-check >> $OUT/slab_rccl_self.jsonl 2>> $OUT/slab.err \
    || { tail $OUT/slab.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sx64 -o run -- \
  python3 scripts/bench_simplex.py --workloads cube --n 64 --lanes 1 --steps 20 > $OUT/simplex64.jsonl 2> $OUT/simplex64.err \
  || { echo "simplex64 rc=$?"; tail $OUT/simplex64.err; exit 1; }
timeout -k 10 300 python scripts/bench_simplex.py --workloads cubetask,cube,fracture --n 16 --steps 200 \
  > $OUT/simplex16.jsonl 2> $OUT/simplex.err || { tail $OUT/simplex.err; exit 1; }
timeout -k 10 300 python scripts/fma_report.py > $OUT/fma_report.jsonl 2> $OUT/fma_report.err || { tail $OUT/fma_report.err; exit 1; }
cat $OUT/fma_report.jsonl
if [ "${PROF:-1}" = 1 ]; then
  TAG=r3${TAG:-end} bash scripts/gpu_profile.sh > $OUT/profile.log 2>&1 || { tail $OUT/profile.log; exit 1; }
  tail -3 $OUT/profile.log
fi
python - <<'EOF' $OUT
import json, sys, glob
o = sys.argv[1]
for f in ("bench_512.json", "bench_256.json"):
    d = json.load(open(f"{o}/{f}"))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["frac"], r["kernel_avg_ms"], r["kernel_symbol"],
          r.get("copy_ceiling", {}).get("GBps"), (d.get("cpu_baseline") or {}).get("value"))
for f in sorted(glob.glob(f"{o}/emulate_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["ms_per_step"], d.get("per_rank_ms_per_step"), d.get("speedup_if_ranks_ran_this_fast_on_K_gpus"))
for f in ("slab.jsonl", "slab_loop64.jsonl", "slab_rccl_self.jsonl"):
    for l in open(f"{o}/{f}"):
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        if "ranks" in d:
            print(f, d["ranks"], d["ms_per_step"], d["kernels"])
for l in open(f"{o}/simplex16.jsonl"):
    d = json.loads(l)
    print("simplex", {k: d[k] for k in d if k in ("workload", "ms_per_step", "value", "vertices")})
EOF
