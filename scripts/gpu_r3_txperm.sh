# GPU session r3: TX lane permutation (tests), then A/B against slots in data-index order.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_txperm_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3_txperm_all.log | head -20; tail -2 gpurun_out/r3_txperm_all.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh default notp default notp
