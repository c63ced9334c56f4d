# GPU session: default bench shape (65536 frames, one pass) vs 78592 frames in two
# pipelined chunks of 39296 (one full decoder generation each), alternating
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in "65536 1" "78592 2"; do
    set -- $cfg
    LTE_PIPELINE_CHUNKS=$2 timeout -k 10 300 python bench.py --frames $1 --steps 5 --warmup 2 --no-cpu > gpurun_out/pf_$1_$2.log 2>&1 || { echo "bench $cfg failed"; tail -3 gpurun_out/pf_$1_$2.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/pf_$1_$2.log').read().strip().splitlines()[-1]); print('F=$1 chunks=$2', d['value'], d['ms_per_step'])"
  done
done
