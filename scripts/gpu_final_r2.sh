# GPU session (round-2 close-out): full gpu test suite, smoke(), default bench
# (f64, with the CPU baseline), and a rocprofv3 kernel-stats profile of it.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_all.log | head -40; tail -3 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_f64.log 2> gpurun_out/bench_f64.err || { echo "bench f64 failed rc=$?"; tail -5 gpurun_out/bench_f64.err; exit 1; }
tail -1 gpurun_out/bench_f64.log | cut -c1-700
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof64 -o run -- python3 bench.py --no-cpu > gpurun_out/prof64.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
tail -1 gpurun_out/prof64.log | cut -c1-300
cut -d, -f1-4 gpurun_out/prof64/run_kernel_stats.csv | head -12
