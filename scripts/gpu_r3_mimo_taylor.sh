# GPU session r3: f64 Taylor Jakes in the multi-antenna channel -- MIMO / velocity parity,
# the whole GPU suite, then every config's throughput.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_tm4.py tests/test_gpu_velocity.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_mt_t.log 2>&1; rc=$?
echo "mimo rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_mt_t.log | head -20; tail -2 gpurun_out/r3_mt_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_mt_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3_mt_all.log | head -20; tail -2 gpurun_out/r3_mt_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python scripts/bench_configs.py --frames 8192 --steps 3 > gpurun_out/r3_configs.jsonl 2> gpurun_out/r3_configs.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_configs.err; exit 1; }
cut -c1-200 gpurun_out/r3_configs.jsonl
