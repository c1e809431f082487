# round-3 final validation (session 2): GPU suite, smoke, the three bench lines, a 2-rank
# self-launched rehearsal, rocprofv3 trace + PMC of the default and C3 rollout launches
set -e
o=gpurun_out/final_s2
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu > $o/bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --no-cpu > $o/bench_wide31.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --no-cpu --steps 1024 > $o/bench_n2_self.log 2>&1
bash tools/profile.sh default_roll_final --steps 640 --warmup 64
bash tools/profile.sh wide31_roll_final --config wide31 --steps 640 --warmup 64
