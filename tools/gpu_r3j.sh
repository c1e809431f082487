set -e
mkdir -p gpurun_out/r3j
timeout -k 10 300 python bench.py > gpurun_out/r3j/bench_default.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --rollout 32 --steps 12 > gpurun_out/r3j/roll_stamps.log 2>&1
bash tools/profile.sh roll_r03 --rollout 32 --steps 640 --warmup 64
