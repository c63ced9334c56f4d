# GPU session: SQ instruction / stall counters per kernel for the config-2
# bench step (65536 frames, one step).  Counters not offered by this
# rocprofv3 are dropped (the list is saved to gpurun_out/pmc_list.txt).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
pass=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU"; do
  pass=$((pass+1)); use=""
  for c in $C; do grep -qw "$c" gpurun_out/pmc_list.txt && use="$use $c"; done
  echo "pass $pass:$use"
  timeout -s KILL 120 rocprofv3 --pmc $use --kernel-trace --output-format csv -d gpurun_out/pmc_sq$pass -o run -- python3 bench.py --frames ${FRAMES:-65536} --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_sq$pass.log 2>&1 || { echo "pmc pass $pass rc=$?"; tail -5 gpurun_out/pmc_sq$pass.log; exit 1; }
done
echo ok
