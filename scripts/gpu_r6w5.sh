set -o pipefail
O=gpurun_out/r6w5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mimo.py tests/test_gpu_philox.py -m gpu -v --timeout 300 --timeout-method thread -k "demap_in_dematch or fused_receiver or fused_simo or frame_tx or wave or sfbc_rx_fused or config4 or simo_symbol or other_config or payload or philox" > $O/tests.log 2>&1; echo "tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests.log | tail -6
for X in 1 0; do LTE_SIMO_XHAND=$X timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu > $O/bench_c3_x$X.json 2> $O/bench_c3_x$X.err && python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('xhand', sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'), d.get('ber_match'))" $O/bench_c3_x$X.json $X; done
bash scripts/gpu_r4.sh r6w5 pmc:3
