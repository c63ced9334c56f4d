# GPU session: full -m gpu suite on the in-tree build, then A/B bench timing
# usage: bash scripts/gpu_ab_full.sh <variant> ...   ("default" = the in-tree build)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash scripts/gpu_ab.sh "$@"
