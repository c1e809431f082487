#!/bin/bash
# A/B the variant libraries on the wide31 bench (C3)
export WAB_DIAGNOSTIC_OK=1  # variant libraries (tools/build_variants.sh) are diagnostic builds
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in 1 2; do
for v in "$@"; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 120 python bench.py --config wide31 --no-cpu --steps 600 --warmup 60 > gpurun_out/ab/w_${v}_$r.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/w_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['roofline']['kernel_us'])"
done; done
