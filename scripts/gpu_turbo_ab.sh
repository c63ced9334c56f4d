# GPU session: turbo parity tests on each library variant, then A/B bench timing
# usage: bash scripts/gpu_turbo_ab.sh <variant> ...   ("default" = the in-tree build)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for V in "$@"; do
  if [ "$V" = default ]; then L=ofdm-lte_amd/lte_phy/liblte_hip.so; else L=ofdm-lte_amd/build/$V/liblte_hip.so; fi
  LTE_HIP_LIB=$L timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "turbo or coded" > gpurun_out/tp_$V.log 2>&1 || { echo "parity $V failed rc=$?"; tail -15 gpurun_out/tp_$V.log; exit 1; }
  echo "$V parity: $(tail -1 gpurun_out/tp_$V.log)"
done
bash scripts/gpu_ab.sh "$@"
