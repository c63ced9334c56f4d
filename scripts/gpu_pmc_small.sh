# GPU session: SQ counters of the small front-end kernels (payload, encode, crc_count) at
# the bench size (65536 frames, one f64 step).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
pass=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  pass=$((pass+1)); use=""
  for c in $C; do grep -qw "$c" gpurun_out/pmc_list.txt && use="$use $c"; done
  echo "pass $pass:$use"
  timeout -s KILL 150 rocprofv3 --pmc $use --kernel-trace --kernel-include-regex 'k_payload|k_encode|k_crc_count' --output-format csv -d gpurun_out/pmcs_$pass -o run -- python3 bench.py --frames 65536 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmcs_$pass.log 2>&1 || { echo "pass $pass rc=$?"; tail -5 gpurun_out/pmcs_$pass.log; exit 1; }
done
echo ok
