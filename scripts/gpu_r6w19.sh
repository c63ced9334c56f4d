# Round 6: wave_symbol_noisy's draw loop unrolled by 2 (build/wsn2) against
# rolled (in-tree) -- configs 3 and 5 (the wave receivers), same box.
set -o pipefail
O=gpurun_out/r6w19; mkdir -p $O
export TMPDIR=/tmp
B=$PWD/ofdm-lte_amd/build
for rep in 1 2; do
for v in u1 wsn2; do
  E=""; [ $v = wsn2 ] && E="LTE_HIP_LIB=$B/wsn2/liblte_hip.so"
  for c in 3 5; do
    env $E timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu > $O/bench_c${c}_${v}_$rep.json 2> $O/bench_c${c}_${v}_$rep.err || { tail -20 $O/bench_c${c}_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c${c}_${v}_$rep.json c$c-$v
  done
done; done
