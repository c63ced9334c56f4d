# Round 6: k_ofdm_txch_flat_w's bin loop rolled (in-tree build) or unrolled by
# 4 / 8 (build/u4, build/u8) against the block kernel (build/mtxold): config 5.
set -o pipefail
O=gpurun_out/r6w14; mkdir -p $O
export TMPDIR=/tmp
B=$PWD/ofdm-lte_amd/build
for rep in 1 2; do
for v in old u1 u4 u8; do
  case $v in old) E="LTE_HIP_LIB=$B/mtxold/liblte_hip.so";; u1) E="";; *) E="LTE_HIP_LIB=$B/$v/liblte_hip.so";; esac
  env $E timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > $O/bench_c5_${v}_$rep.json 2> $O/bench_c5_${v}_$rep.err || { tail -20 $O/bench_c5_${v}_$rep.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c5_${v}_$rep.json c5-$v
done; done
