#!/bin/bash
# per-step time of the rollout line against the launch length T: tools/roll_sweep.sh CONFIG T1 T2 ...
# (WAB_LIB selects a variant library)
set -e
export TMPDIR=/tmp
cfg=$1; shift
mkdir -p gpurun_out/sweep
for T in "$@"; do
  timeout -k 10 200 python bench.py --config $cfg --rollout $T --no-cpu --steps 600 > gpurun_out/sweep/${cfg}_T$T.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/sweep/${cfg}_T$T.log').read().strip().splitlines()[-1]); print('$cfg T=$T', d['ms_per_step']*1e3, 'us/step', d['roofline']['frac'])"
done
