# round 3: full GPU tests, smoke, the default (rollout) bench, the rollout profile
set -e
o=gpurun_out/r3l
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --rollout 32 --steps 12 > $o/roll_stamps.log 2>&1
bash tools/profile.sh roll_r03 --rollout 32 --steps 640 --warmup 64
