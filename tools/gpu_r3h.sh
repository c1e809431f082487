set -e
mkdir -p gpurun_out/r3h
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rollout" > gpurun_out/r3h/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/r3h/bench_step.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --rollout 32 > gpurun_out/r3h/bench_roll32.log 2>&1
timeout -k 10 200 python bench.py --no-cpu --rollout 8 > gpurun_out/r3h/bench_roll8.log 2>&1
