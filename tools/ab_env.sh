#!/bin/bash
# A/B one library under environment settings: tools/ab_env.sh "NAME=VAL ..." "NAME=VAL ..." (default bench, two rounds)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_env
i=0
for r in 1 2; do
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 python bench.py --no-cpu --steps 3000 > gpurun_out/ab_env/v${i}.log 2>&1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_env/v${i}.log').read().strip().splitlines()[-1]); print('$v', $r, d['roofline']['kernel_us'])"
done; done
