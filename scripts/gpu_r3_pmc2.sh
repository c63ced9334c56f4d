# GPU session (round 3, chunked decoder layout): HBM traffic and SQ passes of one
# 8192-frame step, f64 then f32 (scripts/gpu_pmc_r2.sh's passes).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PREC=f64 FRAMES=8192 timeout -k 10 900 bash scripts/gpu_pmc_r2.sh || exit 1
PREC=f32 FRAMES=8192 timeout -k 10 900 bash scripts/gpu_pmc_r2.sh || exit 1
