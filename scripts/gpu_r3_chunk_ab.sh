# GPU session (round 3): decoder block layout chunked over waves (TURBO_CH) and
# nt cache policy -- coded parity on each variant, then interleaved A/B timing.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_turbo_ab.sh default ch32nt ch16nt ch64 || exit 1
bash scripts/gpu_ab.sh default ch32nt ch16nt ch64 default ch32nt
