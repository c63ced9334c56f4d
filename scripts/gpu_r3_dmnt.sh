# GPU session (round 3): non-temporal dematch stores (dmnt1) / + loads (dmnt3) -- coded parity, A/B.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_turbo_ab.sh dmnt1 dmnt3 > /dev/null || exit 1
grep -h passed gpurun_out/tp_dmnt*.log
bash scripts/gpu_ab.sh default dmnt1 dmnt3 default dmnt1 dmnt3
