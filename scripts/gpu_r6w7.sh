set -o pipefail
O=gpurun_out/r6w7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mimo.py tests/test_gpu_philox.py tests/test_gpu_fullsize_mimo.py tests/test_gpu_curve.py -m gpu -q --timeout 300 --timeout-method thread -k "sfbc or config4 or other_config or 4 or transmit_mimo" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
for X in 1 0; do LTE_SFBC_LINK_MERGE=$X timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-shape-ceiling > $O/bench_c4_m$X.json 2> $O/bench_c4_m$X.err && python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('merge', sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms_per_step'))" $O/bench_c4_m$X.json $X; done
bash scripts/gpu_r4.sh r6w7 pmc:4 pmc:5
