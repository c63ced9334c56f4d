# GPU session: default bench (as the driver runs it), kernel-trace stats, then PMC traffic passes (last)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
t0=$(date +%s.%N); timeout -k 10 600 python bench.py > gpurun_out/bench_default_run.log 2> gpurun_out/bench_default_run.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_default_run.err; exit 1; }; echo "bench wall $(python -c "import time; print(round(time.time()-$t0,1))") s"
tail -1 gpurun_out/bench_default_run.err; tail -1 gpurun_out/bench_default_run.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof stats rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/prof_r1/run_kernel_stats.csv | head -8
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$C -o run -- python3 bench.py --frames 8192 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_$C.log 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
  echo "pmc $C ok"; ls gpurun_out/pmc_$C
done
