#!/bin/bash
# One PMC pass of wave-state counters for the step kernel (run via gpurun):
# where wave time goes (active / issue-stalled / parked on waitcnt or barrier) + clock.
# Usage: tools/profile_sq.sh <tag> [bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_state" -o run -- \
  python bench.py --no-cpu --mode launch --steps 40 --warmup 20 "$@" > "$out/bench_state.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python bench.py --no-cpu --mode launch --steps 200 "$@" > "$out/bench_trace.log" 2>&1
echo "profiles in $out"
