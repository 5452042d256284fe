mkdir -p gpurun_out/phys
for args in "--n 512 --steps 10" "--n 512 --steps 10 --maxwell" "--n 256 --steps 10 --layers --no-free" "--n 256 --steps 10 --layers" "--n 256 --steps 10 --no-free" "--n 256 --steps 10 --layers --maxwell --no-free"; do
  timeout -k 10 300 python scripts/bench_physics.py $args >> gpurun_out/phys/phys.jsonl 2>> gpurun_out/phys/phys.err || { echo "fail $args"; tail -3 gpurun_out/phys/phys.err; exit 1; }
done
cat gpurun_out/phys/phys.jsonl
