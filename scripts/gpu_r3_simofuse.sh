# GPU session r3: SIMO receivers in the fused TX channel -- whole GPU suite, SISO/SIMO configs, bench.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_sf_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_sf_all.log | head -20; tail -2 gpurun_out/r3_sf_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --frames 8192 --steps 3 --only c1,c2,c3,c2u,scfdm > gpurun_out/r3_sf.jsonl 2> gpurun_out/r3_sf.err || { echo "configs rc=$?"; tail -5 gpurun_out/r3_sf.err; exit 1; }
python - <<'PY'
import json
for l in open('gpurun_out/r3_sf.jsonl'):
    d=json.loads(l); kk=sorted(d['kernel_ms_per_step'].items(), key=lambda t:-t[1])[:4]
    print(d['config'], d['subframes_per_s'], ', '.join(f'{a} {b:.2f}' for a,b in kk))
PY
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r3_sf_v0.json 2> gpurun_out/r3_sf_v0.err || { echo "v0 rc=$?"; tail -5 gpurun_out/r3_sf_v0.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3_sf_v0.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
