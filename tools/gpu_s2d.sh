# C5 rollout store variants (3 rounds), the per-step C5 profile (returns kernel PMC), C5 rollout profile
set -e
o=gpurun_out/s2d
mkdir -p $o
timeout -k 10 600 bash tools/ab_c5r.sh base fnt1 fnt1ev0 base fnt1 fnt1ev0 > $o/ab_c5r.log 2>&1
bash tools/profile.sh c5_step_s2d --config c5 --rollout 0 --steps 640 --warmup 64
bash tools/profile.sh c5_roll_s2d --config c5 --steps 640 --warmup 64
