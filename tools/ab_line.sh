#!/bin/bash
# A/B one bench line over variant libraries, alternating, R rounds:
#   tools/ab_line.sh OUT R "bench args" v1 v2 ...     (v = product: the in-tree libwab_hip.so;
#   otherwise wab_gym_amd/_lib/var/lib_<v>.so from tools/build_variants.sh or tools/build_rev.sh)
export WAB_DIAGNOSTIC_OK=1  # variant libraries are diagnostic builds
set -eo pipefail
export TMPDIR=/tmp
out=$1; R=$2; args=$3; shift 3
mkdir -p "$out"
for r in $(seq 1 "$R"); do
for v in "$@"; do
  if [ "$v" = product ]; then lib=""; else lib=wab_gym_amd/_lib/var/lib_$v.so; fi
  WAB_LIB=$lib timeout -k 10 200 python bench.py $args --no-cpu --no-extra > "$out/${v}_$r.log" 2>&1 \
    || { tail -20 "$out/${v}_$r.log"; exit 1; }
  python -c "import json; d=json.loads(open('$out/${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, round(d['ms_per_step'] * 1e3, 3), d['roofline'].get('kernel_us'))"
done; done
