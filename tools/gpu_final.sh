# round-end validation on the GPU box: parity tests, smoke, the three bench lines, profiles
set -e
mkdir -p gpurun_out/r2final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2final/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2final/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/r2final/bench_default.log 2>&1
timeout -k 10 200 python bench.py --config wide31 --no-cpu > gpurun_out/r2final/bench_wide31.log 2>&1
bash tools/profile.sh wide_r02b --config wide31 --steps 600 --warmup 60
