# GPU session 5: parity suite; bench default build vs A/B variant builds (LTE_HIP_LIB); kernel-trace stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
summ() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"; }
timeout -k 10 400 python bench.py --frames 32768 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_default.log 2>&1 || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_default.log; exit 1; }
summ gpurun_out/bench_default.log
for V in ${VARIANTS:-plain}; do
  LTE_HIP_LIB=ofdm-lte_amd/build/$V/liblte_hip.so timeout -k 10 400 python bench.py --frames 32768 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_$V.log 2>&1 || { echo "bench $V failed rc=$?"; tail -5 gpurun_out/bench_$V.log; exit 1; }
  summ gpurun_out/bench_$V.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_s5 -o run -- python3 bench.py --frames 32768 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof stats rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/prof_s5/run_kernel_stats.csv
