# GPU session (round 3): chunk sizes 32 / 64 / 128 with nt, other cache-policy
# bits at 32, two waves per SIMD -- coded parity on each, then interleaved A/B.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_turbo_ab.sh ch64nt ch128nt ch32nt3 ch32nt18 ch32nt2w > /dev/null || exit 1
grep -h passed gpurun_out/tp_*.log
bash scripts/gpu_ab.sh ch32nt ch64nt ch128nt ch32nt3 ch32nt18 ch32nt2w ch32nt ch64nt ch128nt
