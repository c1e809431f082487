#!/bin/bash
# A round's closing GPU evidence in one gpurun call (each step under its own time limit, the
# first failure ends it):  tools/final_run.sh OUT_DIR
#   the whole -m gpu suite, smoke(), the driver's bench command, the C3 / C5 / torus / closed-loop C5
#   lines, the per-step ring lines, a 2-rank run sharing the one GPU, the HBM write micro.
set -eo pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/gpu_steps.sh "$out" tests smoke bench bench:wide31 bench:c5 bench:torus mlp ring
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --share-gpu --steps 20 > "$out/bench_n2_share.log" 2>&1 \
  || { tail -30 "$out/bench_n2_share.log"; exit 1; }
tail -c 800 "$out/bench_n2_share.log"
for m in 200 1600; do
  timeout -k 10 60 tools/micro/bin/write_bw $m > "$out/write_bw_${m}MiB.log" 2>&1 || { cat "$out/write_bw_${m}MiB.log"; exit 1; }
done
cat "$out"/write_bw_*.log
