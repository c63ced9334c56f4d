# GPU session r3: multi-antenna channel kernels without the exact-Jakes spill (EX split, f64 J <= 3):
# MIMO parity, then the multi-antenna configs' throughput.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_tm4.py tests/test_gpu_velocity.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_mr_t.log 2>&1; rc=$?
echo "mimo rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_mr_t.log | head -20; tail -2 gpurun_out/r3_mr_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c4,c5,c5r,tm4_sic44,tm4_zf22,tm4_mrc41 > gpurun_out/r3_configs_mimo.jsonl 2> gpurun_out/r3_configs_mimo.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_configs_mimo.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r3_configs_mimo.jsonl'):
    d=json.loads(l); print(d['config'], d['subframes_per_s'], d['ms_per_step'], {k:round(v,2) for k,v in d['kernel_ms_per_step'].items()})
PY
