# GPU session: pipelined-chain parity tests, then A/B of LTE_PIPELINE_CHUNKS on the default bench
# usage: bash scripts/gpu_pipe_ab.sh <chunks> ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
F=${FRAMES:-65536}
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -x -k "pipelined or coded or turbo" > gpurun_out/pipe_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -15 gpurun_out/pipe_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/pipe_tests.log)"
for V in "$@"; do
  LTE_PIPELINE_CHUNKS=$V timeout -k 10 300 python bench.py --frames $F --steps 3 --warmup 1 --no-cpu > gpurun_out/pipe_$V.log 2>&1 || { echo "bench $V failed rc=$?"; tail -5 gpurun_out/pipe_$V.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/pipe_$V.log').read().strip().splitlines()[-1]); print('chunks=$V', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step']['turbo'], d['ber'][10:13])"
done
