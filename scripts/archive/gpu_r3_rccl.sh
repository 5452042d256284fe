#!/bin/bash
# The real RCCL exchange on one GPU (one-rank communicator exchanging with
# itself, gcmx_comm_init(.., 1, 0, 0, 0)): the slab GPU tests, the per-rank
# 64x512x512 step with that exchange in flight, and the copy probe's
# read-only / write-only / copy decomposition.  Output under gpurun_out/r3/rccl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3/${TAG:-rccl}
mkdir -p $OUT
set -o pipefail
[ "${TESTS:-1}" = 1 ] && { timeout -k 10 400 python -u -m pytest tests/test_gpu_slabs.py -x -v --timeout 300 --timeout-method thread -k "rccl or loopback" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }; tail -2 $OUT/pytest.log; }
timeout -k 10 200 python scripts/bench_slab.py --ranks 8,4,2 --steps 30 --rccl-self --no-check > $OUT/slab_rccl_self.jsonl 2> $OUT/slab.err \
  || { tail $OUT/slab.err; exit 1; }
cat $OUT/slab_rccl_self.jsonl
timeout -k 10 200 python scripts/bench_slab.py --ranks 8 --steps 30 --no-check > $OUT/slab_none.jsonl 2>> $OUT/slab.err || { tail $OUT/slab.err; exit 1; }
cat $OUT/slab_none.jsonl
COPY_ONLY=1 timeout -k 10 120 ./tools/copy_probe > $OUT/copy_probe.txt 2>&1 || { cat $OUT/copy_probe.txt; exit 1; }
cat $OUT/copy_probe.txt
