# GPU session (round 3): rocprofv3 --kernel-trace --stats of the default bench, then
# HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) and two SQ passes of one
# 8192-frame f64 step (scripts/gpu_pmc_r2.sh's passes).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_stats -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r3_stats_bench.json 2> gpurun_out/r3_stats_bench.err || { echo "stats rc=$?"; tail -5 gpurun_out/r3_stats_bench.err; exit 1; }
echo "stats ok"; tail -1 gpurun_out/r3_stats_bench.json | cut -c1-300
PREC=f64 FRAMES=8192 timeout -k 10 900 bash scripts/gpu_pmc_r2.sh || exit 1
