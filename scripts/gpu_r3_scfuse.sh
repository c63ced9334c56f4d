# GPU session r3: SC-FDM transmitter with the channel fused -- whole GPU suite, SC-FDM / SISO configs.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_scf_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_scf_all.log | head -20; tail -2 gpurun_out/r3_scf_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only scfdm,c2u,c3 > gpurun_out/r3_scf.jsonl 2> gpurun_out/r3_scf.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_scf.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r3_scf.jsonl'):
    d=json.loads(l); kk=sorted(d['kernel_ms_per_step'].items(), key=lambda t:-t[1])[:4]
    print(d['config'], d['subframes_per_s'], ', '.join(f'{a} {b:.2f}' for a,b in kk))
PY
