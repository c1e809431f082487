# wide rollout: bitmap scrolled in place (no VGPR spills): parity, bench, stamps
set -e
o=gpurun_out/s2n
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "wide_rollout or tiny" -x -q --timeout 300 --timeout-method thread > $o/wide_roll_tests.log 2>&1
timeout -k 10 200 python bench.py --config wide31 --no-cpu > $o/bench_wide31.log 2>&1
timeout -k 10 200 python bench.py --config wide31 --no-cpu > $o/bench_wide31_2.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --config wide31 --rollout 32 --steps 12 > $o/wide_roll_stamps.log 2>&1
