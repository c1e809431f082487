#!/bin/bash
# A/B variant libraries on the per-step wide31 line into a 32-slot obs ring, two rounds:
#   tools/ab_ring.sh v1 v2 ...
export WAB_DIAGNOSTIC_OK=1  # variant libraries (tools/build_variants.sh) are diagnostic builds
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_ring
for r in 1 2; do
for v in "$@"; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --config wide31 --rollout 0 --obs-ring 32 --no-cpu > gpurun_out/ab_ring/${v}_$r.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_ring/${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, round(d['ms_per_step'] * 1e3, 3))"
done; done
