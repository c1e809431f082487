# A/B: wide rollout S after B1; headline obs stores split over three waves
set -e
o=gpurun_out/s2l
mkdir -p $o
WAB_LIB=wab_gym_amd/_lib/var/lib_sb1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "wide_rollout" -x -q --timeout 300 --timeout-method thread > $o/wide_roll_tests_sb1.log 2>&1
WAB_LIB=wab_gym_amd/_lib/var/lib_sw3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "rollout" -x -q --timeout 300 --timeout-method thread > $o/roll_tests_sw3.log 2>&1
WAB_LIB=wab_gym_amd/_lib/var/lib_salign.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "rollout" -x -q --timeout 300 --timeout-method thread > $o/roll_tests_salign.log 2>&1
for r in 1 2; do for v in wbase sb1; do
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --config wide31 --no-cpu --steps 640 > $o/ab_${v}_$r.log 2>&1
python -c "import json; d=json.loads(open('$o/ab_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['ms_per_step'] * 1e3)"
done; done > $o/ab_wide.log
timeout -k 10 600 bash tools/ab_roll.sh sbase sw3 salign > $o/ab_roll.log 2>&1
