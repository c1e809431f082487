# middle-step phase stamps of the C5 and default rollout launches
set -e
o=gpurun_out/s2r
mkdir -p $o
timeout -k 10 300 python tools/phase_stamps.py --no-build --rollout 32 --features --steps 10 > $o/c5_roll_stamps.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --rollout 32 --steps 10 > $o/default_roll_stamps.log 2>&1
