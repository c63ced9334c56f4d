# Round 6: config 3's wave TX with the taps reading x through a 9-register
# window half a symbol at a time (3 waves / SIMD; in-tree, unroll 4; build/h1u2
# unroll 2) against the whole symbol staged (build/full) -- parity, then A/B.
set -o pipefail
O=gpurun_out/r6w17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_philox.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wave_simo or simo_config3 or simo_ref_compat or simo_symbol" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=$PWD/ofdm-lte_amd/build
for rep in 1 2; do
for v in full h1u4 h1u2 block; do
  case $v in full) E="LTE_HIP_LIB=$B/full/liblte_hip.so";; h1u4) E="";; h1u2) E="LTE_HIP_LIB=$B/h1u2/liblte_hip.so";; block) E="LTE_SIMO_TX_WAVE=0";; esac
  env $E timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu > $O/bench_c3_${v}_$rep.json 2> $O/bench_c3_${v}_$rep.err || { tail -20 $O/bench_c3_${v}_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c3_${v}_$rep.json c3-$v
done; done
