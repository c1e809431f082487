# round 3 (session 2): wab_rollout_features parity, C5 rollout bench vs the per-step C5 line,
# A/B of rollout store variants, full GPU suite, 2-rank rehearsal, default bench, C5 profile
set -e
o=gpurun_out/s2c
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k rollout_features -x -v --timeout 200 --timeout-method thread > $o/rf_tests.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu > $o/bench_c5_roll.log 2>&1
timeout -k 10 300 python bench.py --config c5 --rollout 0 --no-cpu > $o/bench_c5_step.log 2>&1
timeout -k 10 600 bash tools/ab_c5r.sh base fnt1 ev0 > $o/ab_c5r.log 2>&1
timeout -k 10 600 bash tools/ab_roll.sh base rnt0 > $o/ab_roll.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --no-cpu --steps 1024 > $o/bench_n2_self.log 2>&1
