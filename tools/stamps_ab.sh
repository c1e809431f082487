# per-phase stamps of stamp-build variants (tools/phase_stamps.py --no-build --lib ...)
set -e
mkdir -p gpurun_out/stamps_ab
cfg=$1; shift
for v in "$@"; do
  timeout -k 10 300 python tools/phase_stamps.py --no-build --lib wab_gym_amd/_lib/var/lib_$v.so --config $cfg --steps 40 > gpurun_out/stamps_ab/${v}_iso.log 2>&1
  timeout -k 10 300 python tools/phase_stamps.py --no-build --lib wab_gym_amd/_lib/var/lib_$v.so --config $cfg --b2b 20 --graph --steps 10 > gpurun_out/stamps_ab/${v}_b2b.log 2>&1
done
