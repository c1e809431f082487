# A/B: staggered first steps of the four workgroups of a CU (rollout builds)
set -e
o=gpurun_out/s2q
mkdir -p $o
for r in 1 2; do for v in sg0 sg1500 sg6000; do
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --no-cpu --steps 3200 > $o/def_${v}_$r.log 2>&1
python -c "import json; d=json.loads(open('$o/def_${v}_$r.log').read().strip().splitlines()[-1]); print('default', '$v', $r, d['ms_per_step'] * 1e3)"
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 640 > $o/c5_${v}_$r.log 2>&1
python -c "import json; d=json.loads(open('$o/c5_${v}_$r.log').read().strip().splitlines()[-1]); print('c5', '$v', $r, d['ms_per_step'] * 1e3)"
done; done > $o/ab_small.log
for r in 1 2; do for v in wg0 wg10000; do
WAB_LIB=wab_gym_amd/_lib/var/lib_$v.so timeout -k 10 200 python bench.py --config wide31 --no-cpu --steps 640 > $o/w_${v}_$r.log 2>&1
python -c "import json; d=json.loads(open('$o/w_${v}_$r.log').read().strip().splitlines()[-1]); print('wide31', '$v', $r, d['ms_per_step'] * 1e3)"
done; done > $o/ab_wide.log
