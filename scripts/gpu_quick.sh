# GPU session: the parity files of the front-end / multi-antenna kernels + per-config throughput (ONLY=c1,c2,...)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_scfdm.py tests/test_gpu_mimo.py tests/test_gpu_tm4.py tests/test_gpu_bf.py} -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_q.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 ${1:+--only $1} > gpurun_out/configs_q.jsonl 2> gpurun_out/configs.err || { echo "configs failed rc=$?"; tail -5 gpurun_out/configs.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/configs_q.jsonl'):
    d=json.loads(l); print(d['config'], d['subframes_per_s'], {k:v for k,v in d['kernel_ms_per_step'].items() if v>0.3})"
