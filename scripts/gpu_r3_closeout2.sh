# GPU session (round 3, after the chunked decoder layout): smoke, the GPU suite,
# the decoder access-shape ceiling of the new layout, and the driver's exact bench
# command under rocprofv3 --kernel-trace --stats.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r3d_smoke.log; exit 1; }
tail -1 gpurun_out/r3d_smoke.log
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 ./scripts/turbo_shape_bench_aux3 > gpurun_out/r3d_shape_aux3.jsonl 2>&1 || { echo "shape rc=$?"; exit 1; }
grep decoder_layout gpurun_out/r3d_shape_aux3.jsonl
t0=$(date +%s)
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d_stats -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3d_driver.json 2> gpurun_out/r3d_driver.err || { echo "driver bench rc=$?"; tail -5 gpurun_out/r3d_driver.err; exit 1; }
echo "driver bench under rocprofv3: wall $(( $(date +%s) - t0 )) s"; tail -1 gpurun_out/r3d_driver.json | cut -c1-300
