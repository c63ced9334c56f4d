# A/B timing of library builds: bash scripts/gpu_ab.sh <variant> ...  ("default" = the in-tree build)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
F=${FRAMES:-65536}
for V in "$@"; do
  if [ "$V" = default ]; then L=ofdm-lte_amd/lte_phy/liblte_hip.so; else L=ofdm-lte_amd/build/$V/liblte_hip.so; fi
  LTE_HIP_LIB=$L timeout -k 10 300 python bench.py --frames $F --steps 3 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/ab_$V.log 2>&1 || { echo "bench $V failed rc=$?"; tail -5 gpurun_out/ab_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_$V.log').read().strip().splitlines()[-1]); print('$V', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
done
