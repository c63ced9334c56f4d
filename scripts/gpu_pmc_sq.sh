# GPU session: SQ instruction / stall counters for the config-2 kernels (one pass)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/pmc_list.txt | sort -u > gpurun_out/sq_counters.txt || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --frames 8192 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_sq.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc_sq.log; exit 1; }
echo ok
