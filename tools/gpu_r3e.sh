set -e
bash tools/profile.sh c5_r03 --config c5 --steps 320 --warmup 64
