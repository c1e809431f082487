"""Per-kernel register and scratch use of the HIP sources (hipcc -Rpass-analysis=kernel-resource-usage),
as a table: python tools/resources.py [source.hip ...] (default: every source of the library)."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(srcs):
    import __graft_entry__ as ge

    if not srcs:
        srcs = [os.path.join(ge.CSRC, s) for s in ge.HIP_SOURCES if s.endswith(".hip") and "capi" not in s]
    for src in srcs:
        r = subprocess.run([ge._hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-c", src,
                            "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
        cur = None
        for line in r.stderr.splitlines():
            m = re.search(r"remark:\s+(Function Name|VGPRs|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2)
            if k == "Function Name":
                if cur:
                    print(cur)
                name = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
                cur = {"kernel": re.sub(r"\(.*", "", name)}
            else:
                cur[k.split(" [")[0]] = v
        if cur:
            print(cur)


if __name__ == "__main__":
    main(sys.argv[1:])
