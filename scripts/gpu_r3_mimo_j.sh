# GPU session r3 (experiment): float64 samples per thread J in the multi-antenna channel kernels
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for j in 1 2 3 5; do
LTE_MJ=$j timeout -k 10 300 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4,c5,c5r > gpurun_out/r3_mj$j.jsonl 2> gpurun_out/r3_mj.err || { echo "rc=$?"; tail -5 gpurun_out/r3_mj.err; exit 1; }
python - $j <<'PY'
import json,sys
for l in open(f'gpurun_out/r3_mj{sys.argv[1]}.jsonl'):
    d=json.loads(l); print('J', sys.argv[1], d['config'], d['subframes_per_s'], 'channel', round(d['kernel_ms_per_step']['channel'],2))
PY
done
