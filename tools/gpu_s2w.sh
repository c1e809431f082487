# the driver's default command on the final tree, and the self-launched 2-rank path
set -e
o=gpurun_out/s2w
mkdir -p $o
timeout -k 10 300 python bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --no-cpu > $o/bench_n2_self.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
