# GPU session: TM4 parity tests + the multi-antenna regression file
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_tm4.py tests/test_gpu_mimo.py -m gpu -q -p no:cacheprovider > gpurun_out/pytest_tm4.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_tm4.log
exit $rc
