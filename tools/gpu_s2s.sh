# C5 rollout: deferred feature rows (W0/W2 slack of the next step) and store unroll A/B; parity
set -e
o=gpurun_out/s2s
mkdir -p $o
for v in f1u1 f1u2 f0u1; do
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rollout_features" -x -q --timeout 200 --timeout-method thread > $o/rf_tests_$v.log 2>&1
done
timeout -k 10 600 bash tools/ab_c5r.sh f0u4 f0u1 f1u1 f1u2 > $o/ab_c5r.log 2>&1
timeout -k 10 300 python tools/phase_stamps.py --no-build --rollout 32 --features --steps 10 > $o/c5_roll_stamps.log 2>&1
