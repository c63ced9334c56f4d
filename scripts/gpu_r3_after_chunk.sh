# GPU session (round 3, chunked decoder layout): every config's throughput
# (f64), the 3 km/h secondary line and the f32 fast-mode line.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 > gpurun_out/r3d_configs.jsonl 2> gpurun_out/r3d_configs.err || { echo "configs failed rc=$?"; tail -5 gpurun_out/r3d_configs.err; exit 1; }
echo configs ok
timeout -k 10 300 python bench.py --velocity 3 --no-cpu > gpurun_out/r3d_v3.json 2> gpurun_out/r3d_v3.err || { echo "v3 rc=$?"; tail -5 gpurun_out/r3d_v3.err; exit 1; }
tail -1 gpurun_out/r3d_v3.json | cut -c1-200
timeout -k 10 300 python bench.py --precision f32 --no-cpu > gpurun_out/r3d_f32.json 2> gpurun_out/r3d_f32.err || { echo "f32 rc=$?"; tail -5 gpurun_out/r3d_f32.err; exit 1; }
tail -1 gpurun_out/r3d_f32.json | cut -c1-200
