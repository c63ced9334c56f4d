# Round 6, config 3's wave-private SIMO receiver, second A/B: per-RE terms in
# LDS; the received samples prefetched one phase ahead or loaded at the symbol start.
set -o pipefail
O=gpurun_out/r6w10; mkdir -p $O
export TMPDIR=/tmp
LTE_HIP_LIB=$PWD/ofdm-lte_amd/build/pf/liblte_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wave_simo or rx_pairs" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EARLY=$PWD/ofdm-lte_amd/build/early/liblte_hip.so
for rep in 1 2; do
for v in pf block early; do
  case $v in pf) E="LTE_SIMO_RX_WAVE=1 LTE_HIP_LIB=$PWD/ofdm-lte_amd/build/pf/liblte_hip.so";; block) E="LTE_SIMO_RX_WAVE=0";; early) E="LTE_SIMO_RX_WAVE=1 LTE_HIP_LIB=$EARLY";; esac
  env $E timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu > $O/bench_c3_${v}_$rep.json 2> $O/bench_c3_${v}_$rep.err || { tail -20 $O/bench_c3_${v}_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms_per_step']['rx_data'])" $O/bench_c3_${v}_$rep.json $v
done; done
