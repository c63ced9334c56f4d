# GPU session: full -m gpu suite, smoke(), default bench (as the driver runs them)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-600
exit $rc
