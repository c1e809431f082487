#!/bin/bash
# One gpurun call's worth of GPU steps (round 4+), each under its own time limit, chained so
# that the first failure ends the call:  tools/gpu_steps.sh OUT_DIR STEP [STEP ...]
#   tests         the whole -m gpu suite (one process)
#   tests:EXPR    the -m gpu tests matching -k EXPR
#   bench         bench.py default line (the driver's command, --steps 20)
#   bench:CONFIG  bench.py --config CONFIG
#   mlp           bench.py --config c5 --policy mlp (closed loop)
#   ring          the per-step launch into a 32-slot obs ring (default and wide31)
#   stamps:ARGS   tools/phase_stamps.py --no-build ARGS (comma-separated)
#   prof:CONFIG   rocprofv3 --kernel-trace --stats of bench.py --config CONFIG
#   smoke         __graft_entry__.smoke()
set -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for s in "$@"; do
  name=${s%%:*}; arg=${s#*:}; [ "$arg" = "$s" ] && arg=""
  echo "== $s $(date +%T)"
  case $name in
    tests)
      if [ -n "$arg" ]; then k=(-k "$arg"); tag=tests_$(echo "$arg" | tr -c 'a-zA-Z0-9_' '_'); else k=(); tag=tests; fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" > "$out/$tag.log" 2>&1 || { tail -30 "$out/$tag.log"; exit 1; }
      tail -3 "$out/$tag.log" ;;
    bench)
      cfg=${arg:-default}
      timeout -k 10 400 python bench.py --config "$cfg" $( [ -z "$arg" ] && echo --steps 20 ) > "$out/bench_$cfg.log" 2>&1 || { tail -30 "$out/bench_$cfg.log"; exit 1; }
      tail -c 600 "$out/bench_$cfg.log" ;;
    mlp)
      timeout -k 10 400 python bench.py --config c5 --policy mlp --no-cpu > "$out/bench_c5_mlp.log" 2>&1 || { tail -30 "$out/bench_c5_mlp.log"; exit 1; }
      tail -c 600 "$out/bench_c5_mlp.log" ;;
    ring)
      for cfg in default wide31; do
        timeout -k 10 300 python bench.py --config $cfg --rollout 0 --obs-ring 32 --no-cpu > "$out/bench_${cfg}_ring.log" 2>&1 || { tail -30 "$out/bench_${cfg}_ring.log"; exit 1; }
        tail -c 300 "$out/bench_${cfg}_ring.log"
      done ;;
    stamps)
      timeout -k 10 300 python tools/phase_stamps.py --no-build ${arg//,/ } > "$out/stamps_${arg//[ ,-]/_}.log" 2>&1 || { tail -30 "$out/stamps_${arg//[ ,-]/_}.log"; exit 1; }
      cat "$out/stamps_${arg//[ ,-]/_}.log" ;;
    prof)
      cfg=${arg:-default}
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$cfg" -o run -- python3 bench.py --config "$cfg" --no-cpu > "$out/prof_$cfg.log" 2>&1 || { tail -30 "$out/prof_$cfg.log"; exit 1; }
      find "$out/prof_$cfg" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$out/prof_$cfg/kernel_stats.csv"
      head -5 "$out/prof_$cfg/kernel_stats.csv" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -30 "$out/smoke.log"; exit 1; }
      cat "$out/smoke.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
