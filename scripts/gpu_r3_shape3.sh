# GPU session (round 3): decoder access shape, cache-policy bits on loads / stores
# (nt) with the wave-chunked row layout, interleaved twice.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for v in "" _aux2 _nl _ns; do
  echo "variant ${v:-base} rep $rep" >> gpurun_out/shape3.jsonl
  timeout -k 10 200 ./scripts/turbo_shape_bench$v >> gpurun_out/shape3.jsonl 2>&1 || { echo "shape$v rc=$?"; exit 1; }
done; done
echo done
