# GPU session r3: fD > 0 taps fused into the SISO TX kernel (per-symbol Taylor sets) --
# whole GPU suite, then the 3 km/h and default bench lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_tv_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_tv_all.log | head -20; tail -2 gpurun_out/r3_tv_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu --velocity 3 > gpurun_out/r3_tv_v3.json 2> gpurun_out/r3_tv_v3.err || { echo "v3 rc=$?"; tail -5 gpurun_out/r3_tv_v3.err; exit 1; }
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r3_tv_v0.json 2> gpurun_out/r3_tv_v0.err || { echo "v0 rc=$?"; tail -5 gpurun_out/r3_tv_v0.err; exit 1; }
python3 - <<'PY'
import json
for f in ('gpurun_out/r3_tv_v3.json','gpurun_out/r3_tv_v0.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], {k:round(v,2) for k,v in d['roofline']['kernel_ms_per_step'].items()})
PY
