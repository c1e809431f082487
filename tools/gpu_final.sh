set -e
mkdir -p gpurun_out/r2final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2final/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2final/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/r2final/bench_default.log 2>&1
timeout -k 10 200 python bench.py --config c5 --no-cpu > gpurun_out/r2final/bench_c5.log 2>&1
bash tools/profile.sh r02_final
