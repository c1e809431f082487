#!/bin/bash
# A/B variant libraries on the rollout bench (T = 32): tools/ab_roll.sh v1 v2 ...
export WAB_DIAGNOSTIC_OK=1  # variant libraries (tools/build_variants.sh) are diagnostic builds
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_roll
for r in 1 2; do
for v in "$@"; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 120 python bench.py --no-cpu --no-extra --no-diag --rollout 64 --steps 3200 > gpurun_out/ab_roll/${v}_$r.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_roll/${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['ms_per_step'] * 1e3)"
done; done
