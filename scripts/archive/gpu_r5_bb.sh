#!/bin/bash
# Round 5, lease BB: the memory side of the placement effect.  TCC->EA read
# requests, their in-flight level (average latency = level / requests) and the
# DRAM credit stalls of the 512^3 step with the layers shuffled (default),
# from one hipMalloc and physically contiguous; a short bench of each first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5/${LEASE:-bb}
mkdir -p $OUT
CT="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
BP="--steps 3 --warmup 1 --reps 1 --no-cpu-baseline --no-profile --no-copy-ceiling --no-clock-probe --no-box-state"
for a in default malloc contiguous; do
  if [ $a = default ]; then E="GCMX_NONE=1"; else E="GCMX_ALLOC=$a"; fi
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 3 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b_$a.json 2> $OUT/b_$a.err || { echo "bench $a rc=$?"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['process_state']['box'].get('unique_id'), d['process_state']['layers']['alloc'])" $OUT/b_$a.json $a
  env $E timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d $OUT/pmc_$a -o run -- python3 bench.py $BP > $OUT/pmc_$a.json 2> $OUT/pmc_$a.err || { echo "pmc $a rc=$?"; tail -3 $OUT/pmc_$a.err; exit 1; }
  echo "pmc $a ok"
done
