# GPU session 4: parity suite after front-end rewrites, bench, kernel-trace stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --frames 32768 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_F32768.log 2>&1 || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_F32768.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_F32768.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], {k: round(v/3,2) for k,v in d['roofline']['kernel_ms'].items()})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_s4 -o run -- python3 bench.py --frames 32768 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof stats rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/prof_s4/run_kernel_stats.csv
