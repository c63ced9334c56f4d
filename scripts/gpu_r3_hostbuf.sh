# GPU session r3: payload bits packed on the device, float64 injections copied straight from the caller --
# whole GPU suite, then the PCIe-inclusive host-buffer throughput.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_hb_all.log 2>&1; rc=$?
echo "all rc=$rc"; grep -E "FAIL|ERROR|assert" gpurun_out/r3_hb_all.log | head -20; tail -2 gpurun_out/r3_hb_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/bench_hostbuf.py --frames 8192 --steps 3 > gpurun_out/r3_hostbuf2.json 2> gpurun_out/r3_hostbuf2.err || { echo "hostbuf rc=$?"; tail -3 gpurun_out/r3_hostbuf2.err; exit 1; }
cat gpurun_out/r3_hostbuf2.json
