# GPU session: selected test files (pass them as arguments; default: every gpu test).
# LTE_TEST_X=1 stops at the first failure.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
X=""; [ "${LTE_TEST_X:-0}" = "1" ] && X="-x"
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -v $X --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sel.log 2>&1; rc=$?; echo "pytest rc=$rc"
grep -E "FAIL|ERROR" gpurun_out/pytest_sel.log | head -60
tail -3 gpurun_out/pytest_sel.log
exit $rc
