# GPU session r3: coding tests (incl. the exact log-MAP coded chain) then the whole GPU suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_coding.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_coding.log 2>&1; rc=$?
echo "coding rc=$rc"; grep -E "logmap|log_map|FAIL|ERROR" gpurun_out/r3_coding.log | head -20; tail -2 gpurun_out/r3_coding.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_all2.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3_all2.log | head -20; tail -2 gpurun_out/r3_all2.log
exit $rc
