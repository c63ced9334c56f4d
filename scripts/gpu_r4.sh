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
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$cfg" -o run -- \
        python3 bench.py --config "$cfg" --gpus 1 --steps 20 --warmup 5 > "$OUT/prof_c$cfg.json" 2> "$OUT/prof_c$cfg.err" \
        || { tail -20 "$OUT/prof_c$cfg.err"; exit 1; }
      cut -c1-300 "$OUT/prof_c$cfg.json" ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
