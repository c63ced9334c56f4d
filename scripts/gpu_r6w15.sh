# Round 6: config 3's wave-private TX (k_ofdm_tx_simo_w) -- SIMO parity tests,
# then a same-box A/B of config 3: tap loop unrolled by 2 (in-tree) or 4
# (build/u4) against the block TX (build/txsold).
set -o pipefail
O=gpurun_out/r6w15; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_velocity.py tests/test_gpu_snr64.py tests/test_gpu_philox.py tests/test_gpu_scfdm.py tests/test_gpu_image.py -m gpu -x -v --timeout 300 --timeout-method thread -k "simo or config3 or c3 or siso or transmit" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=$PWD/ofdm-lte_amd/build
for rep in 1 2; do
for v in old u2 u4; do
  case $v in old) E="LTE_HIP_LIB=$B/txsold/liblte_hip.so";; u2) E="";; u4) E="LTE_HIP_LIB=$B/u4/liblte_hip.so";; esac
  env $E timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu > $O/bench_c3_${v}_$rep.json 2> $O/bench_c3_${v}_$rep.err || { tail -20 $O/bench_c3_${v}_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c3_${v}_$rep.json c3-$v
done; done
