"""Diagnostic: per-phase time of the fused step kernel from in-kernel s_memrealtime stamps.

Builds a separate -DWAB_STAMPS library (never the product build), runs B envs for a few
hundred steps and prints the mean duration of each phase boundary interval over blocks,
plus the launch span (first block start -> last block end).  Shares only; the stamps
themselves cost time.  Usage (GPU box): python tools/phase_stamps.py [--batch 65536] [--config default]
"""
import argparse
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "wab_gym_amd", "_lib", "libwab_hip_stamps.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--config", default="default")
    ap.add_argument("--build-only", action="store_true", help="build the stamps library and exit (CPU side)")
    ap.add_argument("--no-build", action="store_true", help="use the prebuilt stamps library (GPU box)")
    ap.add_argument("--lib", default=OUT, help="the stamps library to load (with --no-build)")
    ap.add_argument("--out", default=OUT, help="where --build-only writes the library")
    ap.add_argument("--cflags", default="", help="extra hipcc flags of the stamps build (A/B variants)")
    ap.add_argument("--b2b", type=int, default=0,
                    help="instead: per-XCD entry/end of the last two of N back-to-back launches")
    ap.add_argument("--rollout", type=int, default=0,
                    help="instead: per-wave phases of the middle step of T-step wab_rollout launches")
    ap.add_argument("--features", action="store_true",
                    help="with --rollout: wab_rollout_features launches (C5), plus the feature emit and row stores")
    ap.add_argument("--graph", action="store_true",
                    help="with --b2b: the N launches captured in a graph and replayed (the bench's shape)")
    args = ap.parse_args()
    import __graft_entry__ as ge

    if not args.no_build:
        src = [os.path.join(ge.CSRC, s) for s in ge.HIP_SOURCES]
        subprocess.run([ge._hipcc()] + [f for f in ge.HIPCC_FLAGS if f != "-DWAB_PRODUCT_BUILD"] + ["-DWAB_STAMPS", "-DWAB_DIAGNOSTIC_BUILD"] + args.cflags.split()
                       + ["-o", args.out] + src, check=True)
    if args.build_only:
        return
    os.environ["WAB_DIAGNOSTIC_OK"] = "1"
    os.environ["WAB_LIB"] = args.lib if args.no_build else OUT
    import numpy as np
    import torch

    import bench
    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    opts, stride, slots, _ = bench.CONFIGS[args.config]
    B = args.batch
    env = BatchedWolvesAndBushesEnv(opts, num_envs=B, device="cuda:0", validate_actions=False,
                                    plane_stride=stride, wolf_slots=slots)
    L = _lib.load()
    L.wab_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    nb = (B + 63) // 64
    st = torch.zeros((nb, 48), dtype=torch.int64, device="cuda:0")
    env.reset()
    L.wab_debug_set_stamps(env._h, st.data_ptr())
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    kind = env.step_kernel
    if args.b2b:
        return b2b_report(env, L, g, args.steps, args.b2b, args.graph)
    if args.rollout:
        if env.step_kernel == "wide":
            return rollout_wide_report(env, st, g, args.steps, args.rollout)
        return rollout_report(env, st, g, args.steps, args.rollout, args.features)
    if kind == "small":
        return small_report(env, st, g, args.steps)
    if kind == "wide":
        return wide_report(env, st, g, args.steps)
    acc, spans, starts, ends, slow_acc = [], [], [], [], []
    sub_acc = {k: [] for k in [(2, 7), (7, 8), (8, 9), (9, 3)]}
    for t in range(args.steps):
        st.zero_()
        env.step(torch.randint(0, env.n_actions, (B,), device="cuda:0", generator=g))
        torch.cuda.synchronize()
        if t < 20:
            continue
        s = st.cpu().numpy().astype(np.int64)
        d = np.diff(s[:, :7], axis=1)  # phase intervals per block (10 ns ticks); order 0..6
        acc.append(d.mean(axis=0))
        spans.append(s[:, 6].max() - s[:, 0].min())
        starts.append(np.percentile(s[:, 0] - s[:, 0].min(), [50, 90, 100]))
        ends.append(np.percentile(s[:, 6] - s[:, 0].min(), [0, 50, 100]))
        ordr = np.argsort(s[:, 6])
        slow = ordr[-len(ordr) // 50:]
        fast = ordr[: len(ordr) // 2]
        slow_acc.append((d[slow].mean(axis=0), d[fast].mean(axis=0),
                         np.bincount(slow % 8, minlength=8), slow[:8]))
        for (a0, a1) in sub_acc:
            sub_acc[(a0, a1)].append((s[:, a1] - s[:, a0]).mean())
    a = np.mean(acc, axis=0) * 10 / 1000
    names = ["A: loads+LDS init", "A2: bitmap scroll", "B|C1: draws | dynamics", "C2|D: plane+stores | resets",
             "E|F1: reset envs | obs stores", "F2: reset obs stores"]
    for n, v in zip(names, a):
        print("%-22s %7.2f us" % (n, v))
    print("%-22s %7.2f us (sum of block means)" % ("block total", a.sum()))
    print("%-22s %7.2f us (first start -> last end)" % ("launch span", np.mean(spans) * 10 / 1000))
    print("block start offsets p50/p90/max (us):", np.round(np.mean(starts, axis=0) * 10 / 1000, 2))
    print("block end times p0/p50/max (us):     ", np.round(np.mean(ends, axis=0) * 10 / 1000, 2))
    print("slowest 2%% blocks, per phase (us):", np.round(np.mean([a for a, _, _, _ in slow_acc], axis=0) * 10 / 1000, 2))
    print("fastest 50%% blocks, per phase (us):", np.round(np.mean([b for _, b, _, _ in slow_acc], axis=0) * 10 / 1000, 2))
    print("slowest blocks by blockIdx%%8:", np.sum([c for _, _, c, _ in slow_acc], axis=0))
    print("example slow block ids:", slow_acc[-1][3])
    # phase C detail: 3 -> 7 -> 8 -> 9 -> 10 -> 11 -> 12 -> 4
    sub = [("C1a: log", 2, 7), ("C1b: wolves", 7, 8), ("C1c: eat", 8, 9), ("C1d: rest+jobs", 9, 3)]
    for n, a0, a1 in sub:
        v = np.mean(sub_acc[(a0, a1)]) * 10 / 1000
        print("  %-20s %7.2f us" % (n, v))


def wide_report(env, st, g, steps):
    """wab_step_wide: wave w stamps 8w + (0 start, 1 before B1, 2 after B1, 3/4 after its P1
    parts, 5 after B2, 6 after its stores retired)."""
    import numpy as np
    import torch

    B = env.num_envs
    nb = (B + 63) // 64
    waves = {"W0 dynamics": ([0, 1, 2, 3, 4, 5, 6], ["loads, despawn, pursuit, grid", "B1 wait", "eat, starve, done",
                                                    "obs issue", "B2 wait", "P2 + drain"]),
             "W1 bushes": ([8, 9, 10, 11, 12, 13, 14], ["bitmap loads, strip, value", "B1 wait", "obs issue",
                                                        "ring B", "B2 wait", "P2 + drain"]),
             "W2 ring": ([16, 17, 18, 19, 20, 21, 22], ["ring A", "B1 wait", "obs issue", "ring B", "B2 wait",
                                                      "P2 + drain"]),
             "W3 ring": ([24, 25, 26, 27, 28, 29, 30], ["ring offsets, ring A", "B1 wait", "obs issue", "ring B",
                                                      "B2 wait", "P2 + drain"])}
    acc = {k: [] for k in waves}
    spans, ends, starts = [], [], []
    for t in range(steps):
        st.zero_()
        env.step(torch.randint(0, env.n_actions, (B,), device="cuda:0", generator=g))
        torch.cuda.synchronize()
        if t < 20:
            continue
        s = st.cpu().numpy().astype(np.int64)[:nb]
        t0 = s[:, [0, 8, 16, 24]].min()
        for k, (cols, _) in waves.items():
            acc[k].append(np.diff(s[:, cols], axis=1).mean(axis=0))
        end = s[:, [6, 14, 22, 30]].max(axis=1)
        spans.append(end.max() - t0)
        ends.append(np.percentile(end - t0, [0, 50, 100]))
        starts.append(np.percentile(s[:, 0] - t0, [0, 50, 90, 100]))
    for k, (cols, names) in waves.items():
        a = np.mean(acc[k], axis=0) * 10 / 1000
        print("%s:" % k)
        for n, v in zip(names, a):
            print("  %-36s %7.2f us" % (n, v))
    print("%-24s %7.2f us (first start -> last end)" % ("launch span", np.mean(spans) * 10 / 1000))
    print("workgroup start p0/p50/p90/max (us):", np.round(np.mean(starts, axis=0) * 10 / 1000, 2))
    print("workgroup end times p0/p50/max (us):", np.round(np.mean(ends, axis=0) * 10 / 1000, 2))
    us = lambda v: np.round(np.asarray(v) * 10 / 1000, 2)  # noqa: E731
    print("W1 P0 detail: start->strip done %.2f, ->rows written %.2f, ->value done %.2f us" % (
        us((s[:, 15] - s[:, 8]).mean()), us((s[:, 31] - s[:, 15]).mean()), us((s[:, 9] - s[:, 31]).mean())))
    e_ = end - t0
    print("last step: end by blockIdx %% 8:", us([e_[np.arange(nb) % 8 == x].mean() for x in range(8)]))
    print("last step: end by blockIdx quartile:", us([q.mean() for q in np.array_split(e_, 4)]))
    obs = s[:, 11] - s[:, 10]
    print("last step: W1 obs issue p0/p50/p90/max:", us(np.percentile(obs, [0, 50, 90, 100])))
    print("last step: W1 obs start (from t0) p0/p50/p90/max:", us(np.percentile(s[:, 10] - t0, [0, 50, 90, 100])))
    order = np.argsort(e_)
    for name, idx in (("fastest 10%", order[: nb // 10]), ("slowest 10%", order[-nb // 10:])):
        print("  %s: obs start %.2f, obs issue %.2f, drain %.2f, end %.2f us" % (
            name, us((s[idx, 10] - t0).mean()), us(obs[idx].mean()), us((s[idx, 14] - s[idx, 13]).mean()), us(e_[idx].mean())))


def b2b_report(env, L, g, steps, n, graph=False):
    """Back-to-back launches as the bench issues them (no synchronisation in between): each
    launch stamps into one of two buffers, alternately; per XCD (the XCC_ID register) the mean
    kernel-entry offset of the last launch's workgroups from its first one, its mean and last
    workgroup end, and the gap from the previous launch's last workgroup end to the first
    entry of the last launch.  Slots: 32 entry, 33 XCC_ID; ends: the small kernel's obs-store
    stamps 6/15/21/27, the wide kernel's 6/14/22/30."""
    import numpy as np
    import torch

    B = env.num_envs
    nb = (B + 63) // 64
    bufs = [torch.zeros((nb, 48), dtype=torch.int64, device="cuda:0") for _ in range(2)]
    ends_cols = [6, 15, 21, 27] if env.step_kernel == "small" else [6, 14, 22, 30]
    acts = torch.randint(0, env.n_actions, (n, B), device="cuda:0", generator=g).to(torch.int8)
    entry, endx, lastx, gaps, spans, karg = [], [], [], [], [], []
    gr = None
    if graph:  # the stamp buffer pointer is a kernel argument: captured per launch
        for i in range(n):  # warm
            env.step(acts[i])
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(gr, stream=side):
                for i in range(n):
                    L.wab_debug_set_stamps(env._h, bufs[i % 2].data_ptr())
                    env.step(acts[i])
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
    for t in range(steps):
        for b in bufs:
            b.zero_()
        torch.cuda.synchronize()
        if gr is not None:
            gr.replay()
        else:
            for i in range(n):
                L.wab_debug_set_stamps(env._h, bufs[i % 2].data_ptr())
                env.step(acts[i])
        torch.cuda.synchronize()
        last = bufs[(n - 1) % 2].cpu().numpy().astype(np.int64)[:nb]
        prev = bufs[(n - 2) % 2].cpu().numpy().astype(np.int64)[:nb]
        t0 = last[:, 32].min()
        xc = last[:, 33] & 7
        end = last[:, ends_cols].max(axis=1) - t0
        entry.append([(last[xc == x, 32] - t0).mean() for x in range(8)])
        endx.append([end[xc == x].mean() for x in range(8)])
        lastx.append([end[xc == x].max() for x in range(8)])
        gaps.append(t0 - prev[:, ends_cols].max())
        if env.step_kernel == "small":
            karg.append([(last[xc == x, 34] - last[xc == x, 32]).mean() for x in range(8)])
        spans.append(end.max())
    us = lambda v: np.round(np.mean(v, axis=0) * 10 / 1000, 2)
    print("back-to-back launches: %d x %d, last two stamped%s" % (steps, n, " (graph replay)" if graph else ""))
    print("entry by XCC, mean (us):   ", us(entry))
    print("end by XCC, mean (us):     ", us(endx))
    print("end by XCC, last (us):     ", us(lastx))
    print("launch span (us):          ", us(spans))
    print("previous last end -> first entry (us):", us(gaps))
    if karg:
        print("entry -> first kernel-argument field by XCC (us):", us(karg))


def rollout_wide_report(env, st, g, launches, T):
    """wab_rollout_wide: the middle step's stamps of each wave (ROLLW_STAMP slots), averaged over
    workgroups and launches; times from the step's first stamp."""
    import numpy as np
    import torch

    B = env.num_envs
    nb = (B + 63) // 64
    seqs = {"W0": [0, 1, 2, 3, 4, 5, 39], "W1": [8, 9, 10, 11, 12], "W2": [16, 17, 18, 19, 20],
            "W3": [24, 25, 26, 27, 28]}
    names = {"W0": ["start", "despawn/pursuit/grid", "emptied clear + log -> B1", "after B1", "eat/done -> B2",
                    "after B2", "P2 + new episodes"],
             "W1": ["start", "scroll (flag)", "tile value", "after B1", "after B2"],
             "W2": ["start", "(step 0: tables)", "stores -> B1", "stores -> B2", "the rest stored"],
             "W3": ["start", "-", "stores -> B1", "stores -> B2", "the rest stored"]}
    acc = {k: [] for k in seqs}
    for it in range(launches):
        st.zero_()
        a = torch.randint(0, env.n_actions, (T, B), device="cuda:0", generator=g).to(torch.int8)
        env.rollout(a)
        torch.cuda.synchronize()
        if it < 3:
            continue
        s = st.cpu().numpy().astype(np.int64)[:nb]
        t0 = s[:, [0, 8, 16, 24]].min(axis=1)
        for k, cols in seqs.items():
            v = s[:, cols]
            ok = (v > 0).all(axis=1)
            acc[k].append((v[ok] - t0[ok, None]).mean(axis=0))
        acc.setdefault("loop", []).append(((s[:, 0] - s[:, 35]).mean(), (s[:, 38] - t0).mean()))
        ent, ex = s[:, 32], s[:, 34]
        xcc = s[:, 33]
        acc.setdefault("xcd", []).append([(ex - ent)[xcc == x].mean() if (xcc == x).any() else 0.0 for x in range(8)])
        acc.setdefault("quart", []).append([q.mean() for q in np.array_split(ex - ent, 8)])
        co = coresidency(s, ent, ex)
        acc.setdefault("cores", []).append(co)
        acc.setdefault("launch", []).append((ex.max() - ent.min(), (ex - ent).mean(), np.percentile(ent - ent.min(), 99),
                                             np.percentile(ex - ent.min(), 1), np.percentile(ex - ent.min(), 50)))
        # the middle step's stamps by dispatch rank on the CU (0..3)
        rk = co[5]
        for k, cols in seqs.items():
            v = s[:, cols]
            ok = (v > 0).all(axis=1)
            acc.setdefault("rank_" + k, []).append(
                [(v[ok & (rk == r)] - t0[ok & (rk == r), None]).mean(axis=0) if (ok & (rk == r)).any()
                 else np.zeros(len(cols)) for r in range(4)])
        acc.setdefault("rank_end", []).append([(s[rk == r, 38] - t0[rk == r]).mean() if (rk == r).any() else 0.0
                                               for r in range(4)])
    for k in seqs:
        a = np.mean(acc["rank_" + k], axis=0) * 10 / 1000
        for r in range(4):
            print("  rank %d %s: %s" % (r, k, ", ".join("%s %.2f" % (n, v) for n, v in zip(names[k], a[r]))))
    print("  middle step: step start -> past its end barrier by rank: %s us"
          % np.round(np.mean(acc["rank_end"], axis=0) * 10 / 1000, 2))
    for k in seqs:
        a = np.mean(acc[k], axis=0) * 10 / 1000
        print("%s: %s" % (k, ", ".join("%s %.2f" % (n, v) for n, v in zip(names[k], a))))
    lp = np.mean(acc["loop"], axis=0) * 10 / 1000
    print("W0: loop top -> its start %.2f us; step start -> past its end barrier %.2f us" % (lp[0], lp[1]))
    la = np.mean(acc["launch"], axis=0) * 10 / 1000
    print("workgroup entry -> exit by XCD (us):", np.round(np.mean(acc["xcd"], axis=0) * 10 / 1000, 1))
    print("workgroup entry -> exit by blockIdx eighth (us):", np.round(np.mean(acc["quart"], axis=0) * 10 / 1000, 1))
    print_coresidency(acc["cores"])
    print("launch: first entry -> last exit %.1f us (%.2f us per step); workgroup entry -> exit mean %.1f us; "
          "entries p99 %.1f us after the first; exits p1 %.1f, p50 %.1f us" % (la[0], la[0] / T, la[1], la[2], la[3], la[4]))


def coresidency(s, ent, ex):
    """Per launch, from the waves' HW_ID (slots 40..43) and the XCD (33): the workgroups of
    each CU ranked by entry (dispatch order); returns durations by rank, by how many other
    groups' W0 share this group's W0 SIMD (0..3), and the SIMD offsets of W1..W3 from W0."""
    import numpy as np

    hw = s[:, 40:44]
    simd = (hw >> 4) & 3
    key = (s[:, 33] << 8) | ((hw[:, 0] >> 8) & 0xFF)
    dur = ex - ent
    by_rank, by_share = [[] for _ in range(8)], [[] for _ in range(4)]
    rank = np.full(len(ent), -1)
    for k in np.unique(key):
        idx = np.nonzero(key == k)[0]
        idx = idx[np.argsort(ent[idx], kind="stable")]
        for r, i in enumerate(idx[:8]):
            by_rank[r].append(dur[i])
            rank[i] = r
            by_share[min(3, int((simd[idx, 0] == simd[i, 0]).sum()) - 1)].append(dur[i])
    offs = np.bincount(((simd[:, 1:] - simd[:, :1]) % 4).ravel(), minlength=4)
    return ([np.mean(v) if v else 0.0 for v in by_rank], [np.mean(v) if v else 0.0 for v in by_share],
            [len(v) for v in by_share], offs, np.bincount(np.bincount(np.unique(key, return_inverse=True)[1])), rank)


def print_coresidency(rows):
    import numpy as np

    print("workgroup entry -> exit by dispatch rank on its CU (us):",
          np.round(np.mean([r[0] for r in rows], axis=0) * 10 / 1000, 1))
    print("  ... by other groups' W0 on its W0's SIMD (0..3):", np.round(np.mean([r[1] for r in rows], axis=0) * 10 / 1000, 1),
          "counts", rows[-1][2])
    print("  W1..W3 SIMD offset from W0 (0..3):", rows[-1][3], "; groups per CU histogram:", rows[-1][4])


def rollout_report(env, st, g, launches, T, features=False):
    """wab_rollout (the small kernel's multi-step build): the middle step's stamps of each wave
    (SMALL_STAMP slots as in small_report; step t > 0 has no loads and no B_init), averaged over
    workgroups and launches; times from the step's first stamp."""
    import numpy as np
    import torch

    B = env.num_envs
    nb = (B + 63) // 64
    seqs = {"W0": [0, 1, 2, 7, 8, 3, 4, 5], "W1": [10, 30, 31, 11, 12, 13, 14],
            "W2": [16, 28, 29, 17, 18, 19, 20], "W3": [22, 23, 24, 9, 25, 26]}
    names = {"W0": ["start", "scroll", "-", "eaten log", "tile value", "eat/starve -> B1", "P1 -> B2", "after B2"],
             "W1": ["start", "B_init", "key", "tile value", "strip", "P1 -> B2", "after B2"],
             "W2": ["start", "B_init", "despawn", "pursuit/grid -> B1", "-", "P1 -> B2", "after B2"],
             "W3": ["start", "spawn set + strip -> B1", "reset draws", "await W1", "new episodes -> B2", "after B2"]}
    acc = {k: [] for k in seqs}
    spans = []
    feats = torch.empty((T, B, 449), device="cuda:0") if features else None
    for it in range(launches):
        st.zero_()
        a = torch.randint(0, env.n_actions, (T, B), device="cuda:0", generator=g).to(torch.int8)
        if features:
            env.rollout_features(a, features=feats)
        else:
            env.rollout(a)
        torch.cuda.synchronize()
        if it < 3:
            continue
        s = st.cpu().numpy().astype(np.int64)[:nb]
        t0 = s[:, [0, 10, 16, 22]].min(axis=1)
        if features:
            acc.setdefault("feat", []).append((s[:, [36, 37]] - t0[:, None]).mean(axis=0))
        for k, cols in seqs.items():
            v = s[:, cols]
            ok = (v > 0).all(axis=1)
            acc[k].append((v[ok] - t0[ok, None]).mean(axis=0))
        spans.append((s[:, [5, 14, 20, 26]].max(axis=1) - t0).mean())
        acc.setdefault("loop", []).append(((s[:, 0] - s[:, 35]).mean(), (s[:, 38] - t0).mean()))
        ent, ex, xcc = s[:, 32], s[:, 39], s[:, 33]
        acc.setdefault("xcd", []).append([(ex - ent)[xcc == x].mean() if (xcc == x).any() else 0.0 for x in range(8)])
        acc.setdefault("eighth", []).append([q.mean() for q in np.array_split(ex - ent, 8)])
        co = coresidency(s, ent, ex)
        acc.setdefault("cores", []).append(co)
        acc.setdefault("launch", []).append((ex.max() - ent.min(), (ex - ent).mean(), np.percentile(ent - ent.min(), 99),
                                             np.percentile(ex - ent.min(), 1), np.percentile(ex - ent.min(), 50)))
        # the middle step's stamps by dispatch rank on the CU (0..3)
        rk = co[5]
        for k, cols in seqs.items():
            v = s[:, cols]
            ok = (v > 0).all(axis=1)
            acc.setdefault("rank_" + k, []).append(
                [(v[ok & (rk == r)] - t0[ok & (rk == r), None]).mean(axis=0) if (ok & (rk == r)).any()
                 else np.zeros(len(cols)) for r in range(4)])
        acc.setdefault("rank_end", []).append([(s[rk == r, 38] - t0[rk == r]).mean() if (rk == r).any() else 0.0
                                               for r in range(4)])
    for k in seqs:
        a = np.mean(acc["rank_" + k], axis=0) * 10 / 1000
        for r in range(4):
            print("  rank %d %s: %s" % (r, k, ", ".join("%s %.2f" % (n, v) for n, v in zip(names[k], a[r]))))
    print("  middle step: step start -> past its end barrier by rank: %s us"
          % np.round(np.mean(acc["rank_end"], axis=0) * 10 / 1000, 2))
    for k in seqs:
        a = np.mean(acc[k], axis=0) * 10 / 1000
        print("%s: %s" % (k, ", ".join("%s %.2f" % (n, v) for n, v in zip(names[k], a))))
    print("step start -> last wave past B2 (mean over workgroups): %.2f us" % (np.mean(spans) * 10 / 1000))
    lp = np.mean(acc["loop"], axis=0) * 10 / 1000
    print("W0: loop top -> its start (parameters, slices) %.2f us; step start -> past its end barrier %.2f us"
          % (lp[0], lp[1]))
    la = np.mean(acc["launch"], axis=0) * 10 / 1000
    print("launch: first entry -> last exit %.1f us (%.2f us per step); workgroup entry -> exit mean %.1f us; "
          "entries p99 %.1f us after the first; exits p1 %.1f, p50 %.1f us" % (la[0], la[0] / T, la[1], la[2], la[3], la[4]))
    print("workgroup entry -> exit by XCD (us):", np.round(np.mean(acc["xcd"], axis=0) * 10 / 1000, 1))
    print("workgroup entry -> exit by blockIdx eighth (us):", np.round(np.mean(acc["eighth"], axis=0) * 10 / 1000, 1))
    print_coresidency(acc["cores"])
    if features:
        f = np.mean(acc["feat"], axis=0) * 10 / 1000
        print("features: emitted %.2f, wave 0's row stores issued %.2f us" % (f[0], f[1]))


def small_report(env, st, g, steps):
    """wab_step_small: W0 stamps 0..9, W1 10..15, W2 16..21, W3 22..27 (SMALL_STAMP)."""
    import numpy as np
    import torch

    B = env.num_envs
    nb = (B + 63) // 64
    waves = {"W0 bushes": ([0, 1, 2, 7, 8, 3, 4, 5, 6],
                           ["loads, scroll, key", "strip draws", "eaten log", "tile value (W1)", "eat, starve",
                            "B1 + status, scalars, bushes", "B2 (+ terminal obs)", "obs stores"]),
             "W1 value + ring A": ([10, 11, 12, 13, 14, 15], ["loads, thresholds, tile value", "ring A",
                                                               "B1 + render S", "B2", "obs stores"]),
             "W2 wolves": ([16, 17, 18, 19, 20, 21], ["loads, despawn, pursuit", "ring B",
                                                       "B1 + spawns, slots, header", "B2", "obs stores"]),
             "W3 ring C": ([22, 23, 25, 26, 27], ["loads, ring C", "B1 + reset draws, new episodes", "B2",
                                                   "obs stores"])}
    acc = {k: [] for k in waves}
    spans, ends = [], []
    by_xcd, slow_w0, fast_w0, start_off, start_xcd, quart = [], [], [], [], [], []
    entry_xcd, first_xcd, w0_lag, xmap = [], [], [], []
    # extra stamps: W2 28 after B_init, 29 after despawn; W1 30 after B_init, 31 after the key;
    # W3 24 after its reset draws, 9 after the wait for W1's (groups without a done env
    # leave 24 and 9 at 0: only groups with one are averaged)
    DETAIL = {"W2 start->B_init": (16, 28), "W2 B_init->despawned": (28, 29), "W2 despawned->grid": (29, 17),
              "W1 start->B_init": (10, 30), "W1 key": (30, 31), "W1 tile value": (31, 11),
              "W0 start->W2 B_init": (0, 28),
              "W3 B1 + reset draws": (23, 24), "W3 await W1": (24, 9), "W3 new episodes": (9, 25)}
    detail = []
    for t in range(steps):
        st.zero_()
        env.step(torch.randint(0, env.n_actions, (B,), device="cuda:0", generator=g))
        torch.cuda.synchronize()
        if t < 20:
            continue
        s = st.cpu().numpy().astype(np.int64)[:nb]
        t0 = min(s[:, 0].min(), s[:, 10].min(), s[:, 16].min(), s[:, 22].min(), s[:, 32].min())
        for k, (cols, _) in waves.items():
            acc[k].append(np.diff(s[:, cols], axis=1).mean(axis=0))
        end = s[:, [6, 15, 21, 27]].max(axis=1)
        spans.append(end.max() - t0)
        ends.append(np.percentile(end - t0, [0, 50, 100]))
        xcd = np.arange(len(end)) % 8
        by_xcd.append([(end - t0)[xcd == x].mean() for x in range(8)])
        start0 = s[:, [0, 10, 16, 22]].min(axis=1) - t0
        start_xcd.append([start0[xcd == x].mean() for x in range(8)])
        quart.append([q.mean() for q in np.array_split(end - t0, 4)])
        xc = s[:, 33] & 7
        entry_xcd.append([(s[xc == x, 32] - t0).mean() for x in range(8)])
        first_xcd.append([(s[xc == x, 32] - t0).min() for x in range(8)])
        w0_lag.append([(s[xc == x, 0] - s[xc == x, 32]).mean() for x in range(8)])
        xmap.append((xc == (np.arange(len(xc)) % 8)).mean())
        order = np.argsort(end)
        cols0 = waves["W0 bushes"][0]
        d0 = np.diff(s[:, cols0], axis=1)
        slow_w0.append(d0[order[-len(order) // 20:]].mean(axis=0))
        fast_w0.append(d0[order[: len(order) // 4]].mean(axis=0))
        start_off.append(((s[:, 0] - t0)[order[-len(order) // 20:]].mean(), (s[:, 0] - t0)[order[: len(order) // 4]].mean()))
        row = []
        for a0, a1 in DETAIL.values():
            ok = (s[:, a0] > 0) & (s[:, a1] > 0)
            row.append((s[ok, a1] - s[ok, a0]).mean() if ok.any() else 0.0)
        detail.append(row)
    for k, (cols, names) in waves.items():
        a = np.mean(acc[k], axis=0) * 10 / 1000
        print("%s:" % k)
        for n, v in zip(names, a):
            print("  %-28s %7.2f us" % (n, v))
    print("detail (us):", ", ".join("%s %.2f" % (n, v * 10 / 1000) for n, v in zip(DETAIL, np.mean(detail, axis=0))))
    print("%-24s %7.2f us (first start -> last end)" % ("launch span", np.mean(spans) * 10 / 1000))
    print("workgroup end times p0/p50/max (us):", np.round(np.mean(ends, axis=0) * 10 / 1000, 2))
    print("mean end time by blockIdx %% 8 (us):", np.round(np.mean(by_xcd, axis=0) * 10 / 1000, 2))
    print("mean start time by blockIdx %% 8 (us):", np.round(np.mean(start_xcd, axis=0) * 10 / 1000, 2))
    print("mean end time by blockIdx quartile (us):", np.round(np.mean(quart, axis=0) * 10 / 1000, 2))
    print("XCC_ID == blockIdx %% 8 for %.1f %% of workgroups" % (100 * np.mean(xmap)))
    print("kernel entry by XCC, first / mean (us):", np.round(np.mean(first_xcd, axis=0) * 10 / 1000, 2),
          np.round(np.mean(entry_xcd, axis=0) * 10 / 1000, 2))
    print("entry -> W0 first stamp by XCC (us):", np.round(np.mean(w0_lag, axis=0) * 10 / 1000, 2))
    print("W0 phases, slowest 5%% of workgroups (us):", np.round(np.mean(slow_w0, axis=0) * 10 / 1000, 2))
    print("W0 phases, fastest 25%% of workgroups (us):", np.round(np.mean(fast_w0, axis=0) * 10 / 1000, 2))
    print("W0 start offset slowest 5%% / fastest 25%% (us):", np.round(np.mean(start_off, axis=0) * 10 / 1000, 2))


if __name__ == "__main__":
    main()
