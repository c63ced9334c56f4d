# GPU session: multi-antenna parity (f64 default + f32 fast mode), then the rest of the GPU suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mimo.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_mimo.log 2>&1; rc=$?
echo "mimo rc=$rc"; grep -E "PASS|FAIL|ERROR|Error" gpurun_out/r3_mimo.log | head -60; tail -3 gpurun_out/r3_mimo.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_mimo.py > gpurun_out/r3_all.log 2>&1; rc2=$?
echo "all rc=$rc2"; grep -E "FAIL|ERROR" gpurun_out/r3_all.log | head -30; tail -3 gpurun_out/r3_all.log
