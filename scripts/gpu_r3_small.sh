# GPU session r3: small-kernel rewrite (payload / crc_count) -- coding + parity tests,
# the whole GPU suite, then a short bench.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_coding.py tests/test_gpu_parity.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_small_t1.log 2>&1; rc=$?
echo "coding+parity rc=$rc"; grep -E "FAIL|ERROR|Error" gpurun_out/r3_small_t1.log | head -20; tail -2 gpurun_out/r3_small_t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_small_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3_small_all.log | head -20; tail -2 gpurun_out/r3_small_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r3_small_bench.json 2> gpurun_out/r3_small_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r3_small_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3_small_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step']); print(d['roofline']['kernel_ms_per_step'])"
