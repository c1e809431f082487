# headline rollout: issue-priority variants (A/B)
set -e
o=gpurun_out/s2x
mkdir -p $o
timeout -k 10 600 bash tools/ab_roll.sh pbase prio2 prio0 > $o/ab_roll.log 2>&1
