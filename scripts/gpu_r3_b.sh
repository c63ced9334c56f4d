# GPU session: fD > 0 chains vs the reference, config-4 BER-curve fixture.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_velocity.py tests/test_gpu_curve.py -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_b.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|ERROR|Error|assert" gpurun_out/r3_b.log | head -60; tail -3 gpurun_out/r3_b.log
exit $rc
