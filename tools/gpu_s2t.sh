set -e
o=gpurun_out/s2t
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "short_segments" -x -v --timeout 200 --timeout-method thread > $o/short_tests.log 2>&1
