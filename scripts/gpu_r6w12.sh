# Round 6: tx_channel's per-RX power partials summed behind one barrier (was
# two per RX) -- the TX parity tests, then a same-box A/B of configs 3 and 2
# against the previous build (build/txold).
set -o pipefail
O=gpurun_out/r6w12; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_philox.py tests/test_gpu_curve.py -m gpu -x -v --timeout 300 --timeout-method thread -k "tx or simo or config3 or c3 or config2 or siso" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OLD=$PWD/ofdm-lte_amd/build/txold/liblte_hip.so
for rep in 1 2; do
for v in new old; do
  E=""; [ $v = old ] && E="LTE_HIP_LIB=$OLD"
  for c in 3 2; do
    env $E timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-shape-ceiling > $O/bench_c${c}_${v}_$rep.json 2> $O/bench_c${c}_${v}_$rep.err || { tail -20 $O/bench_c${c}_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step') or {k: v.get('ms_per_step') for k, v in d['roofline'].get('other_stages', {}).items()})" $O/bench_c${c}_${v}_$rep.json c$c-$v
  done
done; done
