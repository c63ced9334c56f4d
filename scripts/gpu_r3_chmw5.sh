# GPU session (round 3): 2-RX channel kernel at 4 waves/SIMD (103 VGPRs, default)
# vs a 5-wave register cap (g2w5: 96 VGPRs, 24 B scratch) -- config 4 timing.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
LTE_HIP_LIB=ofdm-lte_amd/build/g2w5/liblte_hip.so timeout -k 10 300 python -m pytest tests/test_gpu_mimo.py -m gpu -q -x -p no:cacheprovider > gpurun_out/chm_w5_tests.log 2>&1 || { echo "tests rc=$?"; tail -5 gpurun_out/chm_w5_tests.log; exit 1; }
tail -1 gpurun_out/chm_w5_tests.log
for V in default g2w5 default g2w5; do
  if [ "$V" = default ]; then L=ofdm-lte_amd/lte_phy/liblte_hip.so; else L=ofdm-lte_amd/build/$V/liblte_hip.so; fi
  LTE_HIP_LIB=$L timeout -k 10 300 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4 > gpurun_out/chm_$V.jsonl 2> gpurun_out/chm_$V.err || { echo "$V rc=$?"; tail -5 gpurun_out/chm_$V.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/chm_$V.jsonl'):
    d=json.loads(l); k=d['kernel_ms_per_step']; print('$V', d['config'], round(d['subframes_per_s']), k.get('channel'))
"
done
