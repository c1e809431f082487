set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "headline or c2 or golden or option" > gpurun_out/r3d_tests.log 2>&1
bash tools/ab_env.sh "WAB_WOLF_U32=0" "WAB_WOLF_U32=1"
