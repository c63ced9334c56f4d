# GPU session: throughput of every config (+ TM4 variants)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 ${ONLY:+--only $ONLY} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo "configs failed rc=$?"; tail -5 gpurun_out/configs.err; exit 1; }
cut -c1-260 gpurun_out/configs.jsonl
