# GPU session (round 3): MIMO channel kernels with a 2-RX accumulator group
# (default) vs the 4-RX group (g4) -- multi-antenna parity tests, then config 4
# and TM4 2x2 timing interleaved.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_tests.sh tests/test_gpu_mimo.py tests/test_gpu_tm4.py tests/test_gpu_velocity.py tests/test_gpu_curve.py || exit 1
for V in default g4 default g4; do
  if [ "$V" = default ]; then L=ofdm-lte_amd/lte_phy/liblte_hip.so; else L=ofdm-lte_amd/build/$V/liblte_hip.so; fi
  LTE_HIP_LIB=$L timeout -k 10 300 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4,tm4_zf22 > gpurun_out/chm_$V.jsonl 2> gpurun_out/chm_$V.err || { echo "$V rc=$?"; tail -5 gpurun_out/chm_$V.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/chm_$V.jsonl'):
    d=json.loads(l); k=d['kernel_ms_per_step']; print('$V', d['config'], round(d['subframes_per_s']), k.get('channel'))
"
done
