# GPU session r3: rocprofv3 kernel statistics of the multi-antenna configs (c4, c5, c5r)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in c4 c5 c5r; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3mp_$c -o run -- python3 scripts/bench_configs.py --frames 8192 --steps 2 --only $c > gpurun_out/r3mp_$c.jsonl 2> gpurun_out/r3mp_$c.err || { echo "$c rc=$?"; tail -5 gpurun_out/r3mp_$c.err; exit 1; }
echo "== $c"; python3 - gpurun_out/r3mp_$c/run_kernel_stats.csv <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r['Percentage'])>0.5: print(f"{r['Name'][:70]:70s} {r['Calls']:>4s} {float(r['AverageNs'])/1e6:8.3f} ms {float(r['Percentage']):5.1f}%")
PY
done
