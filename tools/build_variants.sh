#!/bin/bash
# Build A/B variants of the small step kernel into wab_gym_amd/_lib/var/lib_<name>.so (CPU side).
# Usage: tools/build_variants.sh name1 "-DFOO=1 -DBAR=2" name2 "..." ...
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
C=$REPO/wab_gym_amd/csrc
O=/tmp/wab_variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Werror"
mkdir -p $O $REPO/wab_gym_amd/_lib/var
for x in wab_step wab_step_wide wab_features wab_render wab_egocentric wab_capi; do
  fresh=1
  for d in $C/$x.hip $C/*.h $REPO/include/wab.h; do [ $O/$x.o -nt $d ] || fresh=0; done
  [ $fresh = 1 ] || /opt/rocm/bin/hipcc $F -c $C/$x.hip -o $O/$x.o &
done
wait
while [ $# -gt 0 ]; do
  n=$1; d=$2; shift 2
  ( /opt/rocm/bin/hipcc $F $d -c $C/wab_step_small.hip -o $O/small_$n.o &&
    /opt/rocm/bin/hipcc $F -shared -o $REPO/wab_gym_amd/_lib/var/lib_$n.so $O/wab_step.o $O/wab_step_wide.o \
      $O/wab_features.o $O/wab_render.o $O/wab_egocentric.o $O/wab_capi.o $O/small_$n.o ) &
done
wait
ls $REPO/wab_gym_amd/_lib/var
