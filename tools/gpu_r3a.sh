# round 3, first GPU pass: parity tests, smoke, default + C5 bench, the self-launched 2-rank rehearsal
set -e
o=gpurun_out/r3a
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python bench.py --config c5 --no-cpu > $o/bench_c5.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --no-cpu > $o/bench_n2.log 2>&1
