#!/bin/bash
# Build A/B variants of one kernel source (VARIANT_SRC, default wab_step_small) into wab_gym_amd/_lib/var/lib_<name>.so (CPU side).
# Usage: tools/build_variants.sh name1 "-DFOO=1 -DBAR=2" name2 "..." ...
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
C=$REPO/wab_gym_amd/csrc
O=/tmp/wab_variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Werror -DWAB_DIAGNOSTIC_BUILD"  # never the product library (wab_build_guard.h)
mkdir -p $O $REPO/wab_gym_amd/_lib/var
VAR=${VARIANT_SRC:-wab_step_small}   # the source compiled per variant; the others once
ALL="wab_step wab_step_small wab_step_wide wab_features wab_render wab_egocentric wab_torus wab_capi"
COMMON=$(for x in $ALL; do [ $x = $VAR ] || echo $x; done)
for x in $COMMON; do
  fresh=1
  for d in $C/$x.hip $C/*.h $REPO/include/wab.h $REPO/include/wab_torus.h; do [ $O/$x.o -nt $d ] || fresh=0; done
  [ $fresh = 1 ] || /opt/rocm/bin/hipcc $F -c $C/$x.hip -o $O/$x.o &
done
wait
while [ $# -gt 0 ]; do
  n=$1; d=$2; shift 2
  ( /opt/rocm/bin/hipcc $F $d -c $C/$VAR.hip -o $O/${VAR}_$n.o &&
    /opt/rocm/bin/hipcc $F -shared -o $REPO/wab_gym_amd/_lib/var/lib_$n.so $(for x in $COMMON; do echo $O/$x.o; done) \
      $O/${VAR}_$n.o ) &
done
wait
ls $REPO/wab_gym_amd/_lib/var
