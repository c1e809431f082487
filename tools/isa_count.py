"""Static instruction counts of the small step kernel, one wave's path at a time.

Compiles wab_step_small.hip with -DWAB_ONLY_WAVE=k (the other waves' functions dead-code
eliminated; not a runnable build) and counts VALU / SALU / LDS / VMEM instructions of the
default-geometry kernel wab_step_small<8, 11, false, false>, plus the store-only remainder (k = 9).
Loops count once, so this ranks the straight-line cost of each wave's step, the part a
PMC run cannot split by wave.  Usage: python tools/isa_count.py [extra hipcc flags]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "wab_gym_amd", "csrc", "wab_step_small.hip")
KERNEL = os.environ.get("ISA_KERNEL", "_ZN3wab14wab_step_smallILi8ELi11ELb0ELb0EEEvNS_6ParamsE")


def counts(flags):
    out = "/tmp/isa_count.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-DWAB_DIAGNOSTIC_BUILD",
                           "--cuda-device-only", "-S", SRC, "-o", out] + flags, stderr=subprocess.DEVNULL)
    s = open(out).read()
    a = s.index(KERNEL + ":")
    body = s[a:s.index(".Lfunc_end", a)].splitlines()
    c = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0}
    for line in body:
        m = re.match(r"\s+([a-z_0-9]+)", line)
        if not m:
            continue
        op = m.group(1)
        if op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


if __name__ == "__main__":
    extra = sys.argv[1:]
    for k, name in ((0, "W0 bushes"), (1, "W1 draws"), (2, "W2 wolves"), (3, "W3 ring"), (9, "stores only")):
        print("%-12s %s" % (name, counts(["-DWAB_ONLY_WAVE=%d" % k] + extra)))
