#!/bin/bash
# A/B the variant libraries on the standalone featurizer (C5 unfused bench: wab_featurize launch time)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in 1 2; do
for v in "$@"; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 120 python bench.py --config c5 --c5-unfused --no-cpu --steps 640 --warmup 96 > gpurun_out/ab/f_${v}_$r.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/f_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['c5']['featurize_us'])"
done; done
