# GPU session: full -m gpu suite, smoke, per-config throughput, default bench, rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo "configs failed rc=$?"; tail -5 gpurun_out/configs.err; exit 1; }
echo "configs ok"
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo "rocprof ok"
cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | head -8
