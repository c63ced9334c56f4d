# Round-6 close-out: GPU suite, smoke, the driver's bench command (config 2),
# the same under rocprofv3, every config's N = 1 line.  One step per limit.
set -o pipefail
O=${1:-r6fin}
bash scripts/gpu_r4.sh $O suite smoke && \
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$O/bench_driver.json 2> gpurun_out/$O/bench_driver.err && cut -c1-300 gpurun_out/$O/bench_driver.json && \
bash scripts/gpu_r4.sh $O prof:2 bench:3 bench:4 bench:5 bench:5:--channel,rayleigh_mp
