# GPU session r3: compile-time N = 2048 in the multi-antenna TX / RX FFT kernels -- MIMO parity, configs.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_tm4.py tests/test_gpu_velocity.py tests/test_gpu_curve.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_nc_t.log 2>&1; rc=$?
echo "t rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_nc_t.log | head -20; tail -2 gpurun_out/r3_nc_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4,c5,c5r,tm4_sic44,tm4_zf22,tm4_mrc41 > gpurun_out/r3_nc.jsonl 2> gpurun_out/r3_nc.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_nc.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r3_nc.jsonl'):
    d=json.loads(l); kk=sorted(d['kernel_ms_per_step'].items(), key=lambda t:-t[1])[:4]
    print(d['config'], d['subframes_per_s'], ', '.join(f'{a} {b:.2f}' for a,b in kk))
PY
