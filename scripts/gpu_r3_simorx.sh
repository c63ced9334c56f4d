# GPU session r3: fused SIMO MRC receiver -- its parity test, the SIMO / velocity suites, config 3.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "simo or fused" tests/test_gpu_velocity.py tests/test_gpu_curve.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_srx.log 2>&1; rc=$?
echo "t rc=$rc"; grep -E "FAIL|ERROR|assert|Error" gpurun_out/r3_srx.log | head -20; tail -2 gpurun_out/r3_srx.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c3 > gpurun_out/r3_srx.jsonl 2> gpurun_out/r3_srx.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_srx.err; exit 1; }
LTE_PRECISION=f32 timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c3 >> gpurun_out/r3_srx.jsonl 2>> gpurun_out/r3_srx.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_srx.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r3_srx.jsonl'):
    d=json.loads(l); kk=sorted(d['kernel_ms_per_step'].items(), key=lambda t:-t[1])[:4]
    print(d['config'], d['subframes_per_s'], ', '.join(f'{a} {b:.2f}' for a,b in kk))
PY
