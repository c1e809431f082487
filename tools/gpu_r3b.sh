# round 3: wide-kernel spill path (8 register wolf slots + HBM rows): parity, C3 benches
set -e
o=gpurun_out/r3b
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or c3" > $o/gpu_wide_tests.log 2>&1
timeout -k 10 200 python bench.py --config wide31 --no-cpu > $o/bench_wide31_cap32.log 2>&1
timeout -k 10 200 python bench.py --config wide31 --no-cpu --wolf-slots 8 > $o/bench_wide31_cap8.log 2>&1
timeout -k 10 200 python bench.py --config wide31 --no-cpu --wolf-slots 16 > $o/bench_wide31_cap16.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --config wide31 --b2b 20 --graph --steps 10 > $o/wide_b2b_graph.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --config wide31 --steps 40 > $o/wide_isolated.log 2>&1
