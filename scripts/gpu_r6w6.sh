set -o pipefail
O=gpurun_out/r6w6; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_philox.py tests/test_gpu_fullsize_mimo.py -m gpu -q --timeout 300 --timeout-method thread -k "spatial or other_config or 5 or sm_" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
for V in default nostage dspw4; do
  L=ofdm-lte_amd/lte_phy/liblte_hip.so; E=""
  [ $V = dspw4 ] && L=ofdm-lte_amd/build/dspw4/liblte_hip.so
  [ $V = nostage ] && E="LTE_DSP_STAGE=0"
  env $E LTE_HIP_LIB=$L timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5_$V.json 2> $O/bench_c5_$V.err && python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c5_$V.json $V
done
