# GPU session: f64 bench throughput vs frames per step (decoder wave rounds:
# 5 CBs x F/64 waves over 2048 resident waves at 2 waves/SIMD)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for F in ${FRAMES_LIST:-52416 65536 78592 98240}; do
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --frames $F > gpurun_out/frames_$F.log 2> gpurun_out/frames_$F.err || { echo "F=$F failed rc=$?"; tail -3 gpurun_out/frames_$F.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/frames_$F.log').read().strip().splitlines()[-1]);r=d['roofline'];print($F, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['kernel_ms_per_step'].get('ofdm_tx'), r['kernel_ms_per_step'].get('rx_data'))"
done
