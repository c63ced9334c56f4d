# GPU session (round 3 close-out): smoke, the driver's exact bench command, the
# rocprofv3 kernel statistics of the default bench, the 3 km/h and f32 lines,
# then the PMC passes (scripts/gpu_pmc_r2.sh) of one 8192-frame f64 step.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r3f_smoke.log; exit 1; }
tail -1 gpurun_out/r3f_smoke.log
t0=$(date +%s)
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3f_driver.json 2> gpurun_out/r3f_driver.err || { echo "driver bench rc=$?"; tail -5 gpurun_out/r3f_driver.err; exit 1; }
echo "driver bench wall $(( $(date +%s) - t0 )) s"; tail -1 gpurun_out/r3f_driver.json | cut -c1-240
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f_stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r3f_stats_bench.json 2> gpurun_out/r3f_stats.err || { echo "stats rc=$?"; tail -5 gpurun_out/r3f_stats.err; exit 1; }
echo stats ok
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --no-cpu --velocity 3 > gpurun_out/r3f_v3.json 2> gpurun_out/r3f_v3.err || { echo "v3 rc=$?"; tail -5 gpurun_out/r3f_v3.err; exit 1; }
tail -1 gpurun_out/r3f_v3.json | cut -c1-200
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --no-cpu --precision f32 > gpurun_out/r3f_f32.json 2> gpurun_out/r3f_f32.err || { echo "f32 rc=$?"; tail -5 gpurun_out/r3f_f32.err; exit 1; }
tail -1 gpurun_out/r3f_f32.json | cut -c1-200
PREC=f64 FRAMES=8192 timeout -k 10 900 bash scripts/gpu_pmc_r2.sh || exit 1
