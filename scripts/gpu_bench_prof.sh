# GPU session: default bench (as the driver runs it) + rocprofv3 kernel stats of the same command
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | head -6
tail -1 gpurun_out/prof_bench.log | cut -c1-200
