# round 3: C5 profile (returns kernel PMC of the round-3 rewrite), self-launched 2-rank rehearsal
set -e
o=gpurun_out/r3m
mkdir -p $o
bash tools/profile.sh c5_r03b --config c5 --steps 640 --warmup 64
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --no-cpu > $o/bench_n2_self.log 2>&1
timeout -k 10 300 python bench.py --rollout 0 --no-cpu > $o/bench_step.log 2>&1
