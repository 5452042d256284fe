cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r4/alt2; mkdir -p $OUT
for rep in 1 2 3; do for v in alt noalt; do
  GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so timeout -k 10 200 python bench.py --emulate-slabs 8 --steps 10 --reps 3 > $OUT/emu8_${v}_$rep.json 2> $OUT/emu8_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/emu8_${v}_$rep.json'));print('emu8 $v',d['ms_per_step'])"
  GCMX_LIB=gcm_amd/lib/tune/$v/libgcmx.so timeout -k 10 200 python bench.py --n 256 --steps 20 --reps 5 --no-cpu-baseline --no-copy-ceiling > $OUT/b256_${v}_$rep.json 2> $OUT/b256_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b256_${v}_$rep.json'));print('256 $v',d['ms_per_step'],d['roofline']['kernel_avg_ms'])"
done; done
