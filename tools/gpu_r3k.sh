set -e
for v in rs0 rs1 rs2; do
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rollout" > gpurun_out/r3k_tests_$v.log 2>&1
done
bash tools/ab_roll.sh rs0 rs1 rs2
