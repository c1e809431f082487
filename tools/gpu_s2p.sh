# wide rollout: S store timing mixed per CU (A/B), parity of the mixed build
set -e
o=gpurun_out/s2p
mkdir -p $o
WAB_LIB=wab_gym_amd/_lib/var/lib_mix1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "wide_rollout or tiny" -x -q --timeout 300 --timeout-method thread > $o/wide_roll_tests_mix1.log 2>&1
for r in 1 2 3; do for v in mix0 mix1; do
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --config wide31 --no-cpu --steps 640 > $o/ab_${v}_$r.log 2>&1
python -c "import json; d=json.loads(open('$o/ab_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, d['ms_per_step'] * 1e3)"
done; done > $o/ab_wide.log
