#!/bin/bash
# Build the HIP library of a git revision into wab_gym_amd/_lib/var/lib_<name>.so, for A/B
# against the working tree with tools/ab.sh (CPU side).  Usage: tools/build_rev.sh <rev> <name>
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2
W=/tmp/wab_rev_$name
rm -rf $W && mkdir -p $W
git -C $REPO archive $rev wab_gym_amd/csrc include | tar -x -C $W
mkdir -p $REPO/wab_gym_amd/_lib/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -o $REPO/wab_gym_amd/_lib/var/lib_$name.so $W/wab_gym_amd/csrc/*.hip
echo built lib_$name.so from $rev
