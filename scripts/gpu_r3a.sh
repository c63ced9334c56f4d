# GPU session r3a: the driver's exact bench command (f64 headline, with the CPU
# baseline) and the decoder's access-shape microbenchmark.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_driver_cmd.json 2> gpurun_out/r3_driver_cmd.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/r3_driver_cmd.err; exit 1; }
t1=$(date +%s); echo "driver bench wall: $((t1-t0)) s"
tail -1 gpurun_out/r3_driver_cmd.json | cut -c1-900
timeout -k 10 300 ./scripts/turbo_shape_bench > gpurun_out/r3_turbo_shape.json 2>&1 || { echo "shape bench rc=$?"; cat gpurun_out/r3_turbo_shape.json; exit 1; }
cat gpurun_out/r3_turbo_shape.json
