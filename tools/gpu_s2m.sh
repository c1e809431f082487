# rollout edge cases (long eaten logs, log overflow, tiny batch) on both rollout builds; the wide
# rollout's middle-step phase stamps (diagnostic library)
set -e
o=gpurun_out/s2m
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "rollout" -x -v --timeout 300 --timeout-method thread > $o/roll_tests.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --config wide31 --rollout 32 --steps 12 > $o/wide_roll_stamps.log 2>&1
