#!/bin/bash
# A/B the torus variant libraries (tools/build_variants.sh with VARIANT_SRC=wab_torus):
#   tools/ab_torus.sh OUT_DIR variant ...   (bench.py --config torus, two rounds each)
export WAB_DIAGNOSTIC_OK=1  # variant libraries (tools/build_variants.sh) are diagnostic builds
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
for r in 1 2; do
for v in "$@"; do
  lib=wab_gym_amd/_lib/var/lib_$v.so; [ "$v" = base ] && lib=wab_gym_amd/_lib/libwab_hip.so
  WAB_LIB=$lib timeout -k 10 120 python bench.py --config torus --no-cpu --no-diag > "$out/${v}_$r.log" 2>&1
  python -c "import json; d=json.loads(open('$out/${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, round(d['roofline']['kernel_us'] / 64, 2), 'us/turn')"
done; done
