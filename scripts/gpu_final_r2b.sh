# GPU session (round-2 close-out, second pass): full gpu test suite, smoke(),
# the default bench (f64, with the CPU baseline), the f32 fast mode, and a
# rocprofv3 kernel-stats profile of the default bench command.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fin_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/fin_pytest.log | head -20; tail -2 gpurun_out/fin_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/fin_smoke.log; exit 1; }
cat gpurun_out/fin_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/fin_bench64.log 2> gpurun_out/fin_bench64.err || { echo "bench f64 rc=$?"; tail -5 gpurun_out/fin_bench64.err; exit 1; }
tail -1 gpurun_out/fin_bench64.log | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu --precision f32 > gpurun_out/fin_bench32.log 2> gpurun_out/fin_bench32.err || { echo "bench f32 rc=$?"; exit 1; }
tail -1 gpurun_out/fin_bench32.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/fin_prof64 -o run -- python3 bench.py --no-cpu > gpurun_out/fin_prof64.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/fin_prof64/run_kernel_stats.csv | head -14
