# GPU session: LDS / occupancy counters of the front-end kernels on config c2u (uncoded SISO 20 MHz) and c5
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
CFG=${1:-c2u}
for C in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAVES SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_INSTS_VALU" "SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"; do
  tag=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmcl_$tag -o run -- python3 scripts/bench_configs.py --frames 8192 --steps 1 --only $CFG > gpurun_out/pmcl_$tag.log 2>&1 || { echo "pmc $C rc=$?"; tail -5 gpurun_out/pmcl_$tag.log; exit 1; }
  echo "pmc $C ok"
done
