# 64-step rollout lines: the three bench lines and their rocprofv3 + PMC profiles
set -e
o=gpurun_out/s2v
mkdir -p $o
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu > $o/bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --no-cpu > $o/bench_wide31.log 2>&1
bash tools/profile.sh default_roll64 --steps 640 --warmup 64
bash tools/profile.sh c5_roll64 --config c5 --steps 640 --warmup 64
bash tools/profile.sh wide31_roll64 --config wide31 --steps 640 --warmup 64
