set -e
mkdir -p gpurun_out/r3i
for b in 16384 32768 65536; do
timeout -k 10 200 python bench.py --no-cpu --rollout 32 --batch $b --steps 3200 > gpurun_out/r3i/roll_b$b.log 2>&1
python -c "import json; d=json.loads(open('gpurun_out/r3i/roll_b$b.log').read().strip().splitlines()[-1]); print($b, d['ms_per_step'] * 1e3, d['value'])"
done
