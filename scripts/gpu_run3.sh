# GPU session 3: parity suite, bench F sweep, kernel-trace stats, PMC traffic passes (+ calibration)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for F in 32768 65536; do
  timeout -k 10 400 python bench.py --frames $F --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_F$F.log 2>&1 || { echo "bench F=$F failed rc=$?"; tail -5 gpurun_out/bench_F$F.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_F$F.log').read().strip().splitlines()[-1]); print('F=$F', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['kernel_ms'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r1 -o run -- python3 bench.py --frames 32768 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof stats rc=$?"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$C -o run -- ./scripts/pmc_calib > gpurun_out/pmc_calib_$C.log 2>&1 || { echo "calib $C rc=$?"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_bench_$C -o run -- python3 bench.py --frames 32768 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_bench_$C.log 2>&1 || { echo "pmc bench $C rc=$?"; exit 1; }
done
find gpurun_out/prof_r1 gpurun_out/pmc_* -name "*.csv" | head -20
