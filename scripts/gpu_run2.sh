# GPU session 2: parity suite, batch-size sweep, kernel trace
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for F in 8192 16384 32768; do
  timeout -k 10 400 python bench.py --frames $F --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_F$F.log 2>&1 || { echo "bench F=$F failed rc=$?"; tail -5 gpurun_out/bench_F$F.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_F$F.log').read().strip().splitlines()[-1]); print('F=$F', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['kernel_ms'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r1 -- python3 bench.py --frames 16384 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1; echo "rocprof rc=$?"
find gpurun_out/prof_r1 -name "*stats*" | head
