# C3: rollout vs per-step into a 32-slot obs ring (stores reach HBM), plain vs non-temporal obs
set -e
o=gpurun_out/s2g
mkdir -p $o
timeout -k 10 300 python bench.py --config wide31 --rollout 32 --no-cpu > $o/bench_wide31_roll.log 2>&1
WAB_OBS_NT=1 timeout -k 10 300 python bench.py --config wide31 --rollout 32 --no-cpu > $o/bench_wide31_roll_nt.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --rollout 0 --obs-ring 32 --no-cpu > $o/bench_wide31_step_ring.log 2>&1
WAB_OBS_NT=1 timeout -k 10 300 python bench.py --config wide31 --rollout 0 --obs-ring 32 --no-cpu > $o/bench_wide31_step_ring_nt.log 2>&1
timeout -k 10 300 python bench.py --rollout 0 --obs-ring 32 --no-cpu > $o/bench_default_step_ring.log 2>&1
