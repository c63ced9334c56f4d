# GPU session (round 3): decoder access shape in the chunked layout -- checkpoint
# rows per group, a block barrier every 24 steps, cache policy on loads or stores
# only -- interleaved.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in aux3 a3ck1 a3sync l0s3 l3s0 aux3 a3ck1 a3sync; do
  echo "variant $v" >> gpurun_out/shape5.jsonl
  timeout -k 10 200 ./scripts/turbo_shape_bench_$v >> gpurun_out/shape5.jsonl 2>&1 || { echo "shape $v rc=$?"; exit 1; }
done
grep -E "variant|decoder_layout" gpurun_out/shape5.jsonl
