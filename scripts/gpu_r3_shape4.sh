# GPU session (round 3): decoder access shape in the chunked sc0|nt layout --
# reads only (the floor if stores were free), LE rows apart from LS, chunks
# formed per XCD -- interleaved.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in aux3 a3nost a3sep a3xcd aux3 a3xcd a3sep; do
  echo "variant $v" >> gpurun_out/shape4.jsonl
  timeout -k 10 200 ./scripts/turbo_shape_bench_$v >> gpurun_out/shape4.jsonl 2>&1 || { echo "shape $v rc=$?"; exit 1; }
done
grep -E "variant|decoder_layout|\"CH\": 32" gpurun_out/shape4.jsonl
