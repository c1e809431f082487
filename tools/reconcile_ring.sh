#!/bin/bash
# One lease: the per-step ring line (bench.py --rollout 0 --obs-ring 32, graph replays, as the
# driver's configs entry times it) beside rocprofv3 kernel traces of the same command (graph and
# direct launches), the FETCH_SIZE / WRITE_SIZE passes, and the FETCH_SIZE calibration micro.
#   tools/reconcile_ring.sh OUT [bench args...]
set -eo pipefail
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
args="--rollout 0 --obs-ring 32 --no-cpu --no-extra $*"
timeout -k 10 300 python bench.py $args > "$out/bench_line.log" 2>&1 || { tail -20 "$out/bench_line.log"; exit 1; }
tail -c 400 "$out/bench_line.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_graph" -o run -- \
  python3 bench.py $args > "$out/bench_trace_graph.log" 2>&1 || { tail -20 "$out/bench_trace_graph.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py $args --mode launch > "$out/bench_trace.log" 2>&1 || { tail -20 "$out/bench_trace.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- \
  python3 bench.py $args --mode launch --steps 40 --warmup 20 > "$out/bench_fetch.log" 2>&1 || { tail -20 "$out/bench_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- \
  python3 bench.py $args --mode launch --steps 40 --warmup 20 > "$out/bench_write.log" 2>&1 || { tail -20 "$out/bench_write.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_sq" -o run -- \
  python3 bench.py $args --mode launch --steps 40 --warmup 20 > "$out/bench_sq.log" 2>&1 || { tail -20 "$out/bench_sq.log"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/micro_fetch" -o run -- \
  tools/micro/bin/read_bw > "$out/read_bw.log" 2>&1 || { tail -20 "$out/read_bw.log"; exit 1; }
for d in trace_graph trace; do
  f=$(find "$out/$d" -name '*kernel_stats.csv' | head -1); cp "$f" "$out/$d/run_kernel_stats.csv" 2>/dev/null || true
  head -4 "$out/$d/run_kernel_stats.csv"
done
echo done
