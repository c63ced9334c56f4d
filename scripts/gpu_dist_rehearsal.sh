# GPU session: rehearse bench.py's N>1 path on one GPU (2 ranks, gloo backend,
# both ranks on cuda:0): frame-id sharding, barrier, MAX of the elapsed time,
# SUM of the counters, rank-0 JSON line.  Then N=1 with the same frames per rank.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
LTE_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --frames 8192 \
  > gpurun_out/dist2.log 2> gpurun_out/dist2.err || { echo "dist rc=$?"; tail -20 gpurun_out/dist2.err; exit 1; }
tail -1 gpurun_out/dist2.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --frames 8192 --no-cpu > gpurun_out/dist1.log 2> gpurun_out/dist1.err || { echo "n1 rc=$?"; tail -5 gpurun_out/dist1.err; exit 1; }
tail -1 gpurun_out/dist1.log | cut -c1-400
