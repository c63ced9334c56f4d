# GPU session r3: link-noise Philox draws shared by lane pairs -- MIMO tests, config 4 (BER must match the previous run's).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_curve.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_px_t.log 2>&1; rc=$?
echo "t rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_px_t.log | head -20; tail -2 gpurun_out/r3_px_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4 > gpurun_out/r3_px.jsonl 2> gpurun_out/r3_px.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_px.err; exit 1; }
LTE_PRECISION=f32 timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4 > gpurun_out/r3_px32.jsonl 2>> gpurun_out/r3_px.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_px.err; exit 1; }
python - <<'PY'
import json
for f in ('gpurun_out/r3_px.jsonl', 'gpurun_out/r3_px32.jsonl'):
    for l in open(f):
        d=json.loads(l); kk=sorted(d['kernel_ms_per_step'].items(), key=lambda t:-t[1])[:4]
        print(f, d['config'], d['subframes_per_s'], ', '.join(f'{a} {b:.2f}' for a,b in kk)); print(d['ber_by_snr'])
PY
