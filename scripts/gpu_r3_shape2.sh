# GPU session (round 3): decoder access-shape variants (row layout chunked over
# waves, cache-policy bits, reads only), then the GPU test suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "" _aux1 _aux2 _aux3 _aux16 _aux18 _nost; do
  echo "variant ${v:-base}" >> gpurun_out/shape2.jsonl
  timeout -k 10 200 ./scripts/turbo_shape_bench$v >> gpurun_out/shape2.jsonl 2>&1 || { echo "shape$v rc=$?"; exit 1; }
done
cat gpurun_out/shape2.jsonl
bash scripts/gpu_tests.sh
