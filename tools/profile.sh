#!/bin/bash
# Kernel-trace + PMC profiles of bench.py on the GPU box (run via gpurun).
# Usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python bench.py --no-cpu --no-diag --no-extra --mode launch "$@" > "$out/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- \
  python bench.py --no-cpu --no-diag --no-extra --mode launch --steps 40 --warmup 20 "$@" > "$out/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- \
  python bench.py --no-cpu --no-diag --no-extra --mode launch --steps 40 --warmup 20 "$@" > "$out/bench_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_sq" -o run -- \
  python bench.py --no-cpu --no-diag --no-extra --mode launch --steps 40 --warmup 20 "$@" > "$out/bench_sq.log" 2>&1
echo "profiles in $out"
