# GPU session (round 3): the chunked + nt decoder (default) vs sc0|nt (ch32nt3)
# and the contiguous layout (ch1), f64 interleaved, then the f32 fast mode.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_turbo_ab.sh default > /dev/null || exit 1
grep -h passed gpurun_out/tp_default.log
bash scripts/gpu_ab.sh default ch32nt3 ch1 default ch32nt3 default ch32nt3 || exit 1
BENCH_ARGS="--precision f32" bash scripts/gpu_ab.sh ch1 default ch32nt3 ch1 default ch32nt3
