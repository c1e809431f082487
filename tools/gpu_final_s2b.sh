# last check of the committed tree: GPU suite, smoke, default bench line
set -e
o=gpurun_out/final_s2b
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu > $o/bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config wide31 --no-cpu > $o/bench_wide31.log 2>&1
