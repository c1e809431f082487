# rollout length sweep of the default line
set -e
o=gpurun_out/s2u
mkdir -p $o
for r in 1 2; do for T in 16 32 64 128; do
timeout -k 10 200 python bench.py --no-cpu --rollout $T --steps 4096 > $o/T${T}_$r.log 2>&1
python -c "import json; d=json.loads(open('$o/T${T}_$r.log').read().strip().splitlines()[-1]); print('T', $T, $r, d['ms_per_step'] * 1e3, d['roofline']['frac'])"
done; done > $o/sweep.log
