# Round 6, config 3's wave-private SIMO receiver: the 1024-point wave FFT
# microbenchmark, the SIMO parity tests, a same-box A/B of config 3 and its PMC.
set -o pipefail
O=gpurun_out/r6w8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 100 ./scripts/wfft_bench1024 131072 > $O/wfft1024_wpe2.jsonl 2>&1 && \
timeout -k 10 100 ./scripts/wfft_bench1024_wpe3 131072 > $O/wfft1024_wpe3.jsonl 2>&1 || { echo microbench failed; exit 1; }
cat $O/wfft1024_wpe*.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_velocity.py tests/test_gpu_snr64.py tests/test_gpu_philox.py -m gpu -x -v --timeout 300 --timeout-method thread -k "simo or config3 or c3" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for X in 1 0 1; do LTE_SIMO_RX_WAVE=$X timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu > $O/bench_c3_w$X.json 2> $O/bench_c3_w$X.err || { tail -20 $O/bench_c3_w$X.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('wave', sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'), d.get('ber_match',{}).get('frames_identical'))" $O/bench_c3_w$X.json $X; done
bash scripts/gpu_r4.sh r6w8 pmc:3
