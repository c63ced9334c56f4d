# Round 6: config 3 with the wave-private SIMO receiver as the default -- SIMO
# parity tests, one bench line and the PMC summary (profiles/r6_pmc_c3_wave.json).
set -o pipefail
O=gpurun_out/r6w11; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_velocity.py tests/test_gpu_snr64.py tests/test_gpu_philox.py tests/test_roofline_pmc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "simo or config3 or c3 or dry_geometry" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_r4.sh r6w11 bench:3 pmc:3
