#!/bin/bash
# A/B variant libraries (wab_gym_amd/_lib/var/lib_<v>.so) on one bench config, two rounds:
#   tools/ab_bench.sh CONFIG v1 v2 ...   (prints us/step of the line and of the per-step launches)
export WAB_DIAGNOSTIC_OK=1  # variant libraries (tools/build_variants.sh) are diagnostic builds
set -e
export TMPDIR=/tmp
cfg=$1; shift
mkdir -p gpurun_out/ab_bench
for r in 1 2; do
for v in "$@"; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --config $cfg --no-cpu --steps 600 > gpurun_out/ab_bench/${cfg}_${v}_$r.log 2>&1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_bench/${cfg}_${v}_$r.log').read().strip().splitlines()[-1])
ps = d.get('rollout', {}).get('per_step_launch', {})
print('$v', $r, round(d['ms_per_step'] * 1e3, 3), 'per-step ring', ps.get('us_per_step'), 'one buffer', ps.get('one_buffer_us_per_step'))"
done; done
