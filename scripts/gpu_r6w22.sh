# Round 6: config 3's wave TX as one wave per frame with the head samples'
# power fused (k_chan_fix skipped; in-tree) against one wave per symbol
# (build/frame0) and the block TX -- SIMO parity, then A/B.
set -o pipefail
O=gpurun_out/r6w22; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_philox.py tests/test_gpu_velocity.py tests/test_gpu_snr64.py -m gpu -x -v --timeout 300 --timeout-method thread -k "simo or config3 or c3" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=$PWD/ofdm-lte_amd/build
for rep in 1 2; do
for v in frame frame0 block; do
  case $v in frame) E="";; frame0) E="LTE_HIP_LIB=$B/frame0/liblte_hip.so";; block) E="LTE_SIMO_TX_WAVE=0";; esac
  env $E timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 > $O/bench_c3_${v}_$rep.json 2> $O/bench_c3_${v}_$rep.err || { tail -20 $O/bench_c3_${v}_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); bm=d['ber_match']; print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'), bm['frames_identical'], bm['frames'])" $O/bench_c3_${v}_$rep.json c3-$v
done; done
