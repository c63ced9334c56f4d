# GPU session: FETCH_SIZE / WRITE_SIZE passes (one counter per run) of one config-2 bench step
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$C -o run -- python3 bench.py --frames 8192 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -3 gpurun_out/pmc_$C.log; exit 1; }
  echo "pmc $C ok"
done
