# Round 6: config 3 with the wave-private TX and receiver as defaults -- the
# new TX's parity test, one bench line and the PMC (profiles/r6_pmc_c3_wave2.json).
set -o pipefail
O=gpurun_out/r6w16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_roofline_pmc.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wave_simo or dry_geometry" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_r4.sh r6w16 bench:3 pmc:3
