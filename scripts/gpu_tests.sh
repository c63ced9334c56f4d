# GPU session: selected test files (pass them as arguments; default: every gpu test)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest ${@:-tests} -m gpu -q -p no:cacheprovider > gpurun_out/pytest_sel.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_sel.log
exit $rc
