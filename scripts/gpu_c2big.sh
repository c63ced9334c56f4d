# GPU session: full GPU test suite, then config 2 at the bench's 65536 frames per step
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_all.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 65536 --steps 2 --only ${1:-c2} > gpurun_out/c2_65k.jsonl 2> gpurun_out/c2_65k.err || { echo "configs failed"; tail -5 gpurun_out/c2_65k.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c2_65k.jsonl'):
    d=json.loads(l); print(d['config'], d['subframes_per_s'], {k:v for k,v in d['kernel_ms_per_step'].items() if v>0.3})"
