# GPU session r3c: whole GPU suite + smoke on HEAD after the container re-creation.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3c_all.log | head -30; tail -3 gpurun_out/r3c_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/r3c_smoke.log
exit $rc
