# GPU session: A/B of an environment knob on the default bench
# usage: bash scripts/gpu_env_ab.sh VAR v1 v2 ...   (e.g. LTE_TXCH_FUSE 0 1 0 1)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
F=${FRAMES:-65536}; VAR=$1; shift
for V in "$@"; do
  env $VAR=$V timeout -k 10 300 python bench.py --frames $F --steps 3 --warmup 1 --no-cpu > gpurun_out/envab_$V.log 2>&1 || { echo "bench $VAR=$V failed rc=$?"; tail -5 gpurun_out/envab_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/envab_$V.log').read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms_per_step']; print('$VAR=$V', d['value'], d['ms_per_step'], {n: k[n] for n in k if k[n] > 0.3}, d['ber'][9:12])"
done
