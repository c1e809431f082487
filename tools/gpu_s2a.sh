# round 3 (session 2): re-validate the rebuilt tree, C5 profile (returns kernel PMC),
# self-launched 2-rank rehearsal, default bench line
set -e
o=gpurun_out/s2a
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --no-cpu --steps 1024 > $o/bench_n2_self.log 2>&1
bash tools/profile.sh c5_s2a --config c5 --steps 640 --warmup 64
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
