# GPU session: parity suite on the default build and on A/B variants, then A/B timing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest default rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for V in "$@"; do
  LTE_HIP_LIB=ofdm-lte_amd/build/$V/liblte_hip.so timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu_$V.log 2>&1; rc=$?; echo "pytest $V rc=$rc"; tail -4 gpurun_out/pytest_gpu_$V.log
  if [ $rc -gt 1 ]; then exit $rc; fi
done
bash scripts/gpu_ab.sh default "$@"
