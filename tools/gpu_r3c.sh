set -e
o=gpurun_out/r3c
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1
bash tools/ab_env.sh "WAB_WOLF_U32=0" "WAB_WOLF_U32=1"
