set -e
mkdir -p gpurun_out/r3xcd
timeout -k 10 120 tools/micro/bin/xcd_code > gpurun_out/r3xcd/xcd_code.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --b2b 40 --graph --steps 30 > gpurun_out/r3xcd/b2b_graph.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --steps 120 > gpurun_out/r3xcd/isolated.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --wolf-slots 8 --no-cpu > gpurun_out/r3xcd/wide31_slots8.log 2>&1
