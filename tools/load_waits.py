"""List vmcnt waits that split a wave's initial load round trip in the small step kernel.

Every wave of wab_step_small issues all of its loads before its first barrier in one round
trip; a register reuse of a pending load's destination makes the compiler insert an
s_waitcnt vmcnt between two loads, so the loads after it wait for the whole first batch
(a second round trip).  Prints, per s_barrier-delimited region, the waits that sit between
two global loads.  Usage: python tools/load_waits.py [extra hipcc flags]
"""
import re
import subprocess
import sys
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "wab_gym_amd", "csrc", "wab_step_small.hip")
KERNEL = "_ZN3wab14wab_step_smallILi8ELi11ELb0EEEvNS_6ParamsE"


def main(flags):
    out = "/tmp/load_waits.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "--cuda-device-only", "-S", SRC, "-o", out] + flags, stderr=subprocess.DEVNULL)
    s = open(out).read()
    a = s.index(KERNEL + ":")
    body = [l.strip() for l in s[a:s.index(".Lfunc_end", a)].splitlines()
            if l.strip() and not l.strip().startswith(";")]
    bad = 0
    region, loads_seen, pending = 0, 0, []
    for i, l in enumerate(body):
        if l.startswith("s_barrier"):
            region, loads_seen, pending = region + 1, 0, []
        elif l.startswith(("global_load", "buffer_load")):
            if pending:
                for w in pending:
                    print("region %d line %d: %s (then %s)" % (region, w[0], w[1], l))
                    bad += 1
                pending = []
            loads_seen += 1
        elif l.startswith("s_waitcnt") and "vmcnt" in l and loads_seen:
            pending.append((i, l))
    print("%d split round trips" % bad)


if __name__ == "__main__":
    main(sys.argv[1:])
