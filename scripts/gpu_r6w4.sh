set -o pipefail
O=gpurun_out/r6w4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mimo.py tests/test_gpu_philox.py -m gpu -v --timeout 300 --timeout-method thread -k "demap_in_dematch or fused_receiver or fused_simo or frame_tx or wave or sfbc_rx_fused or config4" > $O/tests.log 2>&1; echo "tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests.log | tail -6
LTE_HIP_LIB=ofdm-lte_amd/build/r5lib/liblte_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "fused_simo or fused_receiver" > $O/tests_r5lib.log 2>&1; echo "r5lib rc=$?"; tail -2 $O/tests_r5lib.log
