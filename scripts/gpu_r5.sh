#!/bin/bash
# Round-5 GPU call: bash scripts/gpu_r5.sh OUT STEP...  -- gpu_r4.sh's steps plus
#   ab:<config>:<variant,variant,...>  A/B of library builds on bench.py --config
# (each build from ofdm-lte_amd/build/<variant>/, "default" = the in-tree one).
set -o pipefail
OUT=$1; shift
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p "gpurun_out/$OUT"
for s in "$@"; do
  case ${s%%:*} in
    ab)
      rest=${s#ab:}; cfg=${rest%%:*}; vars=${rest#*:}
      for V in ${vars//,/ }; do
        if [ "$V" = default ]; then L=ofdm-lte_amd/lte_phy/liblte_hip.so; else L=ofdm-lte_amd/build/$V/liblte_hip.so; fi
        echo "== ab c$cfg $V ($(date +%T))"
        LTE_HIP_LIB=$L timeout -k 10 300 python bench.py --config "$cfg" --steps 3 --warmup 1 --no-cpu \
          --no-shape-ceiling > "gpurun_out/$OUT/ab_c${cfg}_$V.json" 2> "gpurun_out/$OUT/ab_c${cfg}_$V.err" \
          || { echo "ab $V failed"; tail -5 "gpurun_out/$OUT/ab_c${cfg}_$V.err"; exit 1; }
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])" "gpurun_out/$OUT/ab_c${cfg}_$V.json" "$V"
      done ;;
    *) bash scripts/gpu_r4.sh "$OUT" "$s" || exit 1 ;;
  esac
done
