set -e
mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_monitor.py -m gpu -x -q --timeout 300 --timeout-method thread -k "returns or monitor" > gpurun_out/r3g/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --config c5 > gpurun_out/r3g/bench_c5.log 2>&1
