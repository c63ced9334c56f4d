# GPU session: parity subset, then the f64 bench with the coded stream staged
# in LDS (default) and gathered through L1/L2 (LTE_TX_STAGE=0)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "signals or fused or coded or simo" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for S in 1 0; do
  LTE_TX_STAGE=$S timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/ab_tx_$S.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/ab_tx_$S.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_tx_$S.log').read().strip().splitlines()[-1]);r=d['roofline'];print('stage=$S', d['value'], r['kernel_ms_per_step'])"
done
