"""Per-wave phase times of the torus kernel's middle turn (a -DWAB2_STAMPS=1 build, results
otherwise as the product's): phase A work and barrier wait, the bush rounds, the mover rounds,
the reward/done pass, the phase-B barrier wait, phase C work and barrier wait, by wave.
    VARIANT_SRC=wab_torus tools/build_variants.sh st "-DWAB2_STAMPS=1"     (here)
    python tools/torus_stamps.py [--lib wab_gym_amd/_lib/var/lib_st.so]     (GPU box)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["A work", "A barrier", "bush (W0-1)", "mover+bush(2-3)", "reward/done", "B barrier", "C work", "C barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="wab_gym_amd/_lib/var/lib_st.so")
    ap.add_argument("--batch", type=int, default=65536)
    args = ap.parse_args()
    os.environ["WAB_DIAGNOSTIC_OK"] = "1"
    os.environ["WAB_LIB"] = args.lib
    import ctypes

    import numpy as np
    import torch

    import bench
    from wab_gym_amd import _lib
    from wab_gym_amd.torus import BatchedWABEnvironment2

    dev = torch.device("cuda:0")
    L = _lib.load()
    B, T = args.batch, 64
    NO, NW, NB = bench.TORUS["counts"]
    env = BatchedWABEnvironment2(bench.TORUS["width"], bench.TORUS["height"], None, NO, NW, NB, num_worlds=B,
                                 seed=0x5EED, device=dev)
    N, R, h = env.N, env.R, env._h
    nblk = -(-B // 64)
    stamps = torch.zeros(nblk * 4 * 16, dtype=torch.int64, device=dev)
    os.environ["WAB2_STAMPS_PTR"] = hex(stamps.data_ptr())
    gen = torch.Generator(device=dev)
    gen.manual_seed(99)
    W = -(-2 * int(env.game_options["max_turns"]) // T) * T
    acts = bench.torus_actions(W + T, B, NO, NW, NB, dev, gen)
    ob = torch.empty((T, B, N, R), dtype=torch.uint8, device=dev)
    rw = torch.empty((T, B, N), dtype=torch.float32, device=dev)
    dn = torch.empty((T, B, N), dtype=torch.uint8, device=dev)
    wr = torch.empty((T, B), dtype=torch.uint8, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for t in range(0, W + T, T):
        if t == W:
            e0.record()
        _lib.check2(L.wab2_rollout(h, acts.data_ptr() + t * B * N, T, ob.data_ptr(), rw.data_ptr(), dn.data_ptr(),
                                   wr.data_ptr(), s), "wab2_rollout")
    e1.record()
    torch.cuda.synchronize()
    us_turn = e0.elapsed_time(e1) * 1e3 / T
    st = stamps.cpu().numpy().reshape(nblk, 4, 16)[:, :, :9].astype(np.float64)
    d = np.diff(st, axis=2)  # [blk][wave][8]
    tot = st[:, :, 8] - st[:, :, 0]
    clk = np.median(tot) / us_turn  # cycles per us (the turn's span over the launch's per-turn time)
    print("launch %.2f us per turn; middle turn spans %.0f cycles (median over waves): %.2f GHz if one turn"
          " = the per-turn mean" % (us_turn, np.median(tot), clk / 1e3))
    print("%-14s %8s %8s %8s %8s   (mean cycles by wave; all waves)" % ("phase", "W0", "W1", "W2", "W3"))
    for k, n in enumerate(NAMES):
        m = d[:, :, k].mean(axis=0)
        print("%-14s %8.0f %8.0f %8.0f %8.0f   %8.0f" % (n, m[0], m[1], m[2], m[3], d[:, :, k].mean()))
    print("%-14s %8.0f %8.0f %8.0f %8.0f" % ("turn", *tot.mean(axis=0)))
    # spread of the workgroups' turn start (how far apart the 4 groups of a CU run)
    start = st[:, 0, 0]
    print("workgroup turn-start spread: p10..p90 %.0f cycles; by blockIdx / 256 (dispatch rank): %s"
          % (np.percentile(start, 90) - np.percentile(start, 10),
             [round(float(np.mean(start[r * 256:(r + 1) * 256] - start.min()))) for r in range(nblk // 256)]))


if __name__ == "__main__":
    main()
