# GPU session: VALU peak microbench, default bench (f64, as the driver runs it),
# the f32 fast mode, and a rocprofv3 kernel-stats profile of the f64 bench.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./scripts/valu_peak_bench > gpurun_out/valu_peak.jsonl 2>&1 || { echo "valu bench failed"; exit 1; }
cat gpurun_out/valu_peak.jsonl
timeout -k 10 600 python bench.py > gpurun_out/bench_f64.log 2> gpurun_out/bench_f64.err || { echo "bench f64 failed rc=$?"; tail -5 gpurun_out/bench_f64.err; exit 1; }
tail -1 gpurun_out/bench_f64.log | cut -c1-600
timeout -k 10 400 python bench.py --precision f32 --no-cpu > gpurun_out/bench_f32.log 2> gpurun_out/bench_f32.err || { echo "bench f32 failed rc=$?"; tail -5 gpurun_out/bench_f32.err; exit 1; }
tail -1 gpurun_out/bench_f32.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof64 -o run -- python3 bench.py --no-cpu > gpurun_out/prof64.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/prof64/run_kernel_stats.csv | head -12
