# GPU session: full gpu test suite, the default bench (f64) and the f32 fast
# mode, and a rocprofv3 kernel-stats profile of the default bench.
# Usage: bash scripts/gpu_check.sh [tag]   (outputs under gpurun_out/<tag>_*)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-chk}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|Error|error" gpurun_out/${T}_pytest.log | head -30; tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${T}_bench64.log 2> gpurun_out/${T}_bench64.err || { echo "bench f64 rc=$?"; tail -5 gpurun_out/${T}_bench64.err; exit 1; }
tail -1 gpurun_out/${T}_bench64.log | cut -c1-260
python - gpurun_out/${T}_bench64.log <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('f64 kernel_ms_per_step', d['roofline'].get('kernel_ms_per_step'))
EOF
timeout -k 10 300 python bench.py --no-cpu --precision f32 > gpurun_out/${T}_bench32.log 2> gpurun_out/${T}_bench32.err || { echo "bench f32 rc=$?"; tail -5 gpurun_out/${T}_bench32.err; exit 1; }
tail -1 gpurun_out/${T}_bench32.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_prof64 -o run -- python3 bench.py --no-cpu > gpurun_out/${T}_prof64.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cut -d, -f1-4 gpurun_out/${T}_prof64/run_kernel_stats.csv | head -14
