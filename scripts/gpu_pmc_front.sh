# GPU session: per-kernel HBM bytes (FETCH_SIZE, WRITE_SIZE in separate passes) + kernel trace for the config-2 bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmcf_$C -o run -- python3 bench.py --frames 8192 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmcf_$C.log 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
  echo "pmc $C ok"
done
