# GPU session: -m gpu suite, smoke, per-config throughput, default bench,
# rocprofv3 kernel stats, then the PMC traffic passes (FETCH_SIZE, WRITE_SIZE;
# one counter per pass) on the config-2 bench at 8192 frames
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo "configs failed rc=$?"; tail -5 gpurun_out/configs.err; exit 1; }
echo "configs ok"
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo "rocprof ok"; cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | head -6
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$C -o run -- python3 bench.py --frames 8192 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_$C.log 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
  echo "pmc $C ok"
done
