#!/bin/bash
# A/B variant libraries on the C5 rollout bench (wab_rollout_features, T = 32): us per step
export WAB_DIAGNOSTIC_OK=1  # variant libraries (tools/build_variants.sh) are diagnostic builds
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_c5r
for r in 1 2; do
for v in "$@"; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 150 python bench.py --config c5 --no-cpu --steps 640 --warmup 96 > gpurun_out/ab_c5r/${v}_$r.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_c5r/${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['ms_per_step'] * 1e3)"
done; done
