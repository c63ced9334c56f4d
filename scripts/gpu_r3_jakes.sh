# GPU session r3: Taylor-expanded Jakes taps (fD > 0) -- the 3 km/h parity tests, the
# whole GPU suite, then the 3 km/h and default bench lines.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_velocity.py tests/test_gpu_mimo.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_jk_t.log 2>&1; rc=$?
echo "velocity+mimo rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_jk_t.log | head -20; tail -2 gpurun_out/r3_jk_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_jk_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3_jk_all.log | head -20; tail -2 gpurun_out/r3_jk_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --no-cpu --velocity 3 > gpurun_out/r3_jk_v3.json 2> gpurun_out/r3_jk_v3.err || { echo "v3 rc=$?"; tail -5 gpurun_out/r3_jk_v3.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3_jk_v3.json').read().strip().splitlines()[-1])
print('v3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
