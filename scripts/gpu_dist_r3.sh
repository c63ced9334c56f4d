# GPU session (round 3): bench.py's N>1 path as the driver starts it (self-launch via
# torch.distributed.run, one process per rank) rehearsed on one GPU with gloo (RCCL
# refuses two ranks on one device): 2 ranks on cuda:0, cpu_baseline from the launcher
# parent, roofline over both ranks' timers.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
LTE_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --steps 3 --warmup 1 --frames 16384 --cpu-seconds 5 \
  > gpurun_out/r3_dist2.json 2> gpurun_out/r3_dist2.err || { echo "dist rc=$?"; tail -20 gpurun_out/r3_dist2.err; exit 1; }
tail -1 gpurun_out/r3_dist2.json | cut -c1-600
