# GPU session (round 2): HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per
# pass) of one bench step (PREC=f64 default), then two SQ passes (instruction
# mix, LDS, waits) of the same step.  Counters this
# rocprofv3 does not offer are dropped (list in gpurun_out/pmc_list.txt).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
FR=${FRAMES:-8192}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${PREC:-f64}_$C -o run -- python3 bench.py --frames $FR --steps 1 --warmup 0 --no-cpu --precision ${PREC:-f64} > gpurun_out/pmc_${PREC:-f64}_$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -3 gpurun_out/pmc_${PREC:-f64}_$C.log; exit 1; }
  echo "pmc $C ok"
done
pass=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
  pass=$((pass+1)); use=""
  for c in $C; do grep -qw "$c" gpurun_out/pmc_list.txt && use="$use $c"; done
  echo "sq pass $pass:$use"
  timeout -s KILL 150 rocprofv3 --pmc $use --kernel-trace --output-format csv -d gpurun_out/pmc_${PREC:-f64}_sq$pass -o run -- python3 bench.py --frames $FR --steps 1 --warmup 0 --no-cpu --precision ${PREC:-f64} > gpurun_out/pmc_${PREC:-f64}_sq$pass.log 2>&1 || { echo "sq pass $pass rc=$?"; tail -5 gpurun_out/pmc_${PREC:-f64}_sq$pass.log; exit 1; }
done
echo ok
