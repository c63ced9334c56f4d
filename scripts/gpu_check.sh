cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 gfx > gpurun_out/arch.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then timeout -k 10 400 python bench.py --steps 3 --warmup 1 --frames 4096 --cpu-seconds 10 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -5 gpurun_out/bench.log; fi
