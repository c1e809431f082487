set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3f
for v in 0 1; do
WAB_RETURNS_VEC1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/trace_v$v -o run -- python bench.py --no-cpu --config c5 --steps 320 --warmup 64 > gpurun_out/r3f/bench_v$v.log 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "returns" > gpurun_out/r3f/tests.log 2>&1
