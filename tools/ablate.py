"""Cost attribution for the small step kernel: build variant libraries that skip one piece of
work (results are wrong; barriers, flags and control flow are kept), then time them against
the full kernel with tools/ab.sh on the GPU box.  The delta of a variant is what that piece
costs inside the whole launch (contention included), which per-wave stamps cannot show.

CPU side: python tools/ablate.py [name ...]  -> wab_gym_amd/_lib/var/lib_x_<name>.so
The edits are applied to a copy of the sources in /tmp; the product sources are untouched.
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "wab_gym_amd", "csrc")

# name -> [(old, new)] applied to wab_step_small.hip
ABLATIONS = {
    "full": [],
    # the entering-strip draws (W1 + W3): no hashing
    "nostrip": [("  if (h.dir != DIR_STAY) {\n    const bool horiz", "  if (false) {\n    const bool horiz")],
    # the obs stores after B2
    "nostore": [("    store_obs(p, lds + L.stream, threadIdx.x);", "    if (p.B < 0) store_obs(p, lds + L.stream, threadIdx.x);")],
    # despawn draws (W2): every wolf kept, no hashing
    "nodespawn": [("      if (!live4) continue;\n      uint32_t h1[4], hh[4], ts[4];",
                   "      if (live4 || !live4) { keep |= live4 << g4; continue; }\n      uint32_t h1[4], hh[4], ts[4];")],
    # the reset draws of the done envs (W1 + W3 reset_chunk)
    "noresetdraws": [("  for (int j4 = 0; j4 < n_jobs; j4 += 4) {\n    uint32_t kb0[4], h1[4], hb[4];",
                      "  for (int j4 = 0; j4 < n_jobs * 0; j4 += 4) {\n    uint32_t kb0[4], h1[4], hb[4];")],
    # pursuit, wolf grid and kill (W2)
    "nopursuit": [("    if (!((live >> g4) & 0xFu)) continue;\n#pragma unroll\n    for (int q = 0; q < 4; ++q) {\n      const int k = g4 + q;\n      const bool on",
                   "    if (true) continue;\n#pragma unroll\n    for (int q = 0; q < 4; ++q) {\n      const int k = g4 + q;\n      const bool on")],
    # the eaten-log scan (W0)
    "nolog": [("  for (int k = 0; k < 4; ++k) {\n    const bool in = i0 + k < ne;", "  for (int k = 0; k < 4 * 0; ++k) {\n    const bool in = i0 + k < ne;")],
    # rendering S into the bit-stream (W1)
    "norender": [("    render_s(p, s, lane, info);\n  }\n  SMALL_STAMP(13);", "    if (p.B < 0) render_s(p, s, lane, info);\n  }\n  SMALL_STAMP(13);")],
    # the new episodes (W3)
    "nonewep": [("      if (job) new_episode<SLOTS>(p, s, h, g, j, (uint32_t)lane * (uint32_t)p.OB, wolf_of);",
                 "      if (job && p.B < 0) new_episode<SLOTS>(p, s, h, g, j, (uint32_t)lane * (uint32_t)p.OB, wolf_of);")],
    # the ostrich tile's generated value (W1)
    "nocval": [("  s.cval[lane] =\n      (uint32_t)bush_value_fast(", "  s.cval[lane] = 0u *\n      (uint32_t)bush_value_fast(")],
    # the ring's spawn set (W3)
    "nospawn": [("  if (p.wolves_on && h.active)\n    spawn_hits(s.gap, p.R,", "  if (p.wolves_on && h.active && p.B < 0)\n    spawn_hits(s.gap, p.R,")],
}


def build(name):
    tmp = "/tmp/wab_ablate_%s" % name
    shutil.rmtree(tmp, ignore_errors=True)
    csrc = os.path.join(tmp, "wab_gym_amd", "csrc")
    shutil.copytree(CSRC, csrc)
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
    f = os.path.join(csrc, "wab_step_small.hip")
    s = open(f).read()
    for old, new in ABLATIONS[name]:
        assert s.count(old) == 1, (name, old[:60], s.count(old))
        s = s.replace(old, new)
    open(f, "w").write(s)
    os.makedirs(os.path.join(REPO, "wab_gym_amd", "_lib", "var"), exist_ok=True)
    out = os.path.join(REPO, "wab_gym_amd", "_lib", "var", "lib_x_%s.so" % name)
    srcs = [os.path.join(csrc, x) for x in sorted(os.listdir(csrc)) if x.endswith(".hip")]
    return subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                             "-ffp-contract=off", "-o", out] + srcs)


if __name__ == "__main__":
    names = sys.argv[1:] or list(ABLATIONS)
    procs = [build(n) for n in names]
    assert all(p.wait() == 0 for p in procs)
    print("built", " ".join("x_" + n for n in names))
