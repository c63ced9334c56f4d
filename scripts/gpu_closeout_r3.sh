# GPU session (round 3 close-out): the driver's exact bench command under
# rocprofv3 --kernel-trace --stats, so the committed kernel statistics and the
# bench line (roofline.avg_launch_ms) come from one run.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/r3c_smoke.log; exit 1; }
tail -1 gpurun_out/r3c_smoke.log
t0=$(date +%s)
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c_stats -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_driver.json 2> gpurun_out/r3c_driver.err || { echo "driver bench rc=$?"; tail -5 gpurun_out/r3c_driver.err; exit 1; }
echo "driver bench under rocprofv3: wall $(( $(date +%s) - t0 )) s"; tail -1 gpurun_out/r3c_driver.json | cut -c1-300
find gpurun_out/r3c_stats -name "*kernel_stats.csv" | head -5
