#!/bin/bash
# A/B the current library against a previous round's (ABI 2) build in wab_gym_amd/_lib/var/lib_r2.so
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_r2
for r in 1 2; do
  WAB_LIB=wab_gym_amd/_lib/var/lib_r2.so timeout -k 10 120 python -c "
import sys, runpy
sys.argv = ['bench.py', '--no-cpu', '--steps', '3000']
import ctypes
import wab_gym_amd._lib as L
L.ABI_VERSION = 2
class _Old(ctypes.CDLL):  # the previous round's library lacks this round's new symbols
    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return type('Missing', (), {})()
ctypes.CDLL = _Old
runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab_r2/r2_$r.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/ab_r2/r2_$r.log').read().strip().splitlines()[-1]); print('r2', $r, d['roofline']['kernel_us'])"
  for v in 0; do
    WAB_WOLF_U32=$v timeout -k 10 120 python bench.py --no-cpu --steps 3000 > gpurun_out/ab_r2/u32_${v}_$r.log 2>&1
    python -c "import json; d=json.loads(open('gpurun_out/ab_r2/u32_${v}_$r.log').read().strip().splitlines()[-1]); print('cur u32=$v', $r, d['roofline']['kernel_us'])"
  done
done
