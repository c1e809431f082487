#!/bin/bash
# The round's profile set (tools/profile.sh per line), chained: the first failure ends the call.
#   tools/profile_set.sh ROUND name ...   names: default, ring, torus, wide31, wide31_ring, c5
set -e
r=$1; shift
for n in "$@"; do
  case $n in
    default) bash tools/profile.sh ${r}_default --steps 640 ;;
    ring) bash tools/profile.sh ${r}_default_ring32 --rollout 0 --obs-ring 32 ;;
    torus) bash tools/profile.sh ${r}_torus --config torus ;;
    wide31) bash tools/profile.sh ${r}_wide31 --config wide31 ;;
    wide31_ring) bash tools/profile.sh ${r}_wide31_ring32 --config wide31 --rollout 0 --obs-ring 32 ;;
    c5) bash tools/profile.sh ${r}_c5 --config c5 ;;
    *) echo "unknown profile $n"; exit 2 ;;
  esac
done
