#!/bin/bash
# Round-4 GPU steps, parameterised: bash scripts/gpu_r4.sh OUT STEP [STEP ...]
#   tests:<pytest-args>  pytest (-m gpu) on the given files / -k expression
#   suite                the whole GPU suite
#   bench:<config>[:<extra bench.py args, comma-separated>]
#   prof:<config>        bench under rocprofv3 --kernel-trace --stats
#   smoke                __graft_entry__.smoke()
# Every step runs under its own time limit; the first failure ends the script.
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
for s in "$@"; do
  kind=${s%%:*}
  arg=${s#*:}
  [ "$arg" = "$s" ] && arg=""
  echo "== $s ($(date +%T))"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest ${arg//,/ } -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/tests_${arg//[^a-zA-Z0-9]/_}.log" 2>&1 || { tail -30 "$OUT/tests_${arg//[^a-zA-Z0-9]/_}.log"; exit 1; }
      tail -3 "$OUT/tests_${arg//[^a-zA-Z0-9]/_}.log" ;;
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/suite.log" 2>&1 || { tail -30 "$OUT/suite.log"; exit 1; }
      tail -3 "$OUT/suite.log" ;;
    bench)
      cfg=${arg%%:*}
      extra=${arg#*:}
      [ "$extra" = "$arg" ] && extra=""
      tag=c${cfg}${extra//[^a-zA-Z0-9]/_}
      timeout -k 10 600 python bench.py --config "$cfg" ${extra//,/ } > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" \
        || { tail -20 "$OUT/bench_$tag.err"; exit 1; }
      cat "$OUT/bench_$tag.json" | cut -c1-400 ;;
    prof)
      cfg=${arg%%:*}
      extra=${arg#*:}
      [ "$extra" = "$arg" ] && extra=""
      tag=c${cfg}${extra//[^a-zA-Z0-9]/_}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$tag" -o run -- \
        python3 bench.py --config "$cfg" --gpus 1 --steps 20 --warmup 5 ${extra//,/ } > "$OUT/prof_$tag.json" \
        2> "$OUT/prof_$tag.err" || { tail -20 "$OUT/prof_$tag.err"; exit 1; }
      cut -c1-300 "$OUT/prof_$tag.json"
      f=$(find "$OUT/prof_$tag" -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && cp "$f" "$OUT/kstats_$tag.csv" && head -12 "$OUT/kstats_$tag.csv" | cut -d, -f1-4 ;;
    pmc)
      # SQ instruction / stall counters (2 passes) and HBM bytes (FETCH_SIZE,
      # WRITE_SIZE: one pass each) of one step, every counter pass its own run
      cfg=${arg%%:*}
      extra=${arg#*:}
      [ "$extra" = "$arg" ] && extra=""
      tag=c${cfg}${extra//[^a-zA-Z0-9]/_}
      i=0
      for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
               "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU" \
               "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/pmc_${tag}_p$i" -o run -- \
          python3 bench.py --config "$cfg" --steps 1 --warmup 0 --no-cpu ${extra//,/ } > "$OUT/pmc_${tag}_p$i.log" 2>&1 \
          || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc_${tag}_p$i.log"; exit 1; }
      done
      echo "pmc $tag: $i passes" ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
