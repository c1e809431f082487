# wide rollout with the on-chip eaten log: parity; C3 rollout vs per-step (one obs buffer, and a
# 32-slot obs ring whose stores reach HBM as the rollout's do)
set -e
o=gpurun_out/s2f
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "wide_rollout" -x -v --timeout 300 --timeout-method thread > $o/wide_roll_tests.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --rollout 32 --no-cpu > $o/bench_wide31_roll.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --rollout 0 --obs-ring 32 --no-cpu > $o/bench_wide31_step_ring.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --rollout 0 --no-cpu > $o/bench_wide31_step.log 2>&1
timeout -k 10 300 python bench.py --rollout 0 --obs-ring 32 --no-cpu > $o/bench_default_step_ring.log 2>&1
