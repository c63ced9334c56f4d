# Round 6: config 5's TX + flat links as one wave per (frame, RX)
# (k_ofdm_txch_flat_w) -- MIMO parity tests, then a same-box A/B of config 5
# against the previous build (build/mtxold) and its PMC.
set -o pipefail
O=gpurun_out/r6w13; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_philox.py tests/test_gpu_fullsize_mimo.py tests/test_gpu_tm4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "spatial or wave or config5 or tm4 or flat or other_config" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OLD=$PWD/ofdm-lte_amd/build/mtxold/liblte_hip.so
for rep in 1 2; do
for v in new old; do
  E=""; [ $v = old ] && E="LTE_HIP_LIB=$OLD"
  env $E timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5_${v}_$rep.json 2> $O/bench_c5_${v}_$rep.err || { tail -20 $O/bench_c5_${v}_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c5_${v}_$rep.json c5-$v
done; done
bash scripts/gpu_r4.sh r6w13 pmc:5
