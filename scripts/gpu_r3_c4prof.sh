# GPU session (round 3): kernel statistics of config 4 (SFBC 2x2 + turbo) and config 5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_prof_$c -o run -- python3 scripts/bench_configs.py --frames 8192 --steps 3 --only $c > gpurun_out/r3_prof_$c.jsonl 2> gpurun_out/r3_prof_$c.err || { echo "$c rc=$?"; tail -5 gpurun_out/r3_prof_$c.err; exit 1; }
  python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/r3_prof_$c/run_kernel_stats.csv')))
for r in rows[:12]: print('$c', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), r['Percentage'])
"
done
