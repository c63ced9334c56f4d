# GPU session: config-2 throughput vs frames per step
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for F in ${FRAMES_LIST:-32768 49152 65536 98304}; do
  timeout -k 10 300 python bench.py --frames $F --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_F$F.log 2> gpurun_out/bench_F$F.err || { echo "F=$F failed rc=$?"; tail -3 gpurun_out/bench_F$F.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/bench_F$F.log').read().strip().splitlines()[-1]); r=d['roofline']
print($F, d['value'], d['ms_per_step'], r['avg_launch_ms'], {k:v for k,v in r['kernel_ms_per_step'].items() if v>0.5})"
done
