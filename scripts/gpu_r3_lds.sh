# GPU session r3 (LDS): whole GPU suite, a short bench, and the LDS counters of
# one f64 bench step (bank-conflict cycles per LDS instruction per kernel).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_lds_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/r3_lds_tests.log | head -20; tail -2 gpurun_out/r3_lds_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r3_lds_bench.json 2> gpurun_out/r3_lds_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r3_lds_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3_lds_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step']); print(d['roofline']['kernel_ms_per_step'])"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_lds_f64 -o run -- python3 bench.py --frames 8192 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_lds_f64.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc_lds_f64.log; exit 1; }
echo pmc ok
