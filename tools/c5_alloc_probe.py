"""Probe: the sharded C5 rollout (bench.py --config c5) timed as bench.py's `configs` entry
times it, with the rollout buffers allocated in different ways, to find why the `configs` entry
and the C5 line's own run differ.  Usage (GPU box):
    python tools/c5_alloc_probe.py [--prealloc-gb G] [--zeros] [--config c5|wide31]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prealloc-gb", type=float, default=0.0)
    ap.add_argument("--zeros", action="store_true")
    ap.add_argument("--free-gb", type=float, default=0.0, help="allocate, zero and free this much first")
    ap.add_argument("--config", default="c5", help="comma-separated: timed in turn in one process")
    ap.add_argument("--seed", type=int, default=4321)
    ap.add_argument("--offset-kb", type=int, default=-1, help="features/planes at this offset (KiB) past a 1 GiB boundary")
    args = ap.parse_args()
    import torch

    import bench
    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    L = _lib.load()
    dev = torch.device("cuda:0")
    if args.free_gb > 0:
        x = torch.zeros(int(args.free_gb * 2**30), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        del x
        torch.cuda.empty_cache()
    for cfg in args.config.split(","):
        one(args, cfg, torch, bench, _lib, L, BatchedWolvesAndBushesEnv, dev)
        torch.cuda.empty_cache()


def one(args, cfg, torch, bench, _lib, L, BatchedWolvesAndBushesEnv, dev):
    B, T, S, NL = 65536, 64, 2, 32
    Bs = B // S
    opts, stride, slots, _ = bench.CONFIGS[cfg]
    keep = None
    if args.prealloc_gb > 0:
        keep = torch.zeros(int(args.prealloc_gb * 2**30), dtype=torch.uint8, device=dev)
    alloc = torch.zeros if args.zeros else torch.empty
    envs = [BatchedWolvesAndBushesEnv(opts, num_envs=Bs, seed=0x5EED, device=dev, env_id_base=k * Bs, autoreset=True,
                                      validate_actions=False, plane_stride=stride, wolf_slots=slots) for k in range(S)]
    for e in envs:
        e.reset()
    e0 = envs[0]
    W = -(-2 * int(e0.game_options["max_turns"]) // T) * T
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed)
    acts = torch.randint(0, e0.n_actions, (W + NL * T, B), device=dev, generator=gen).to(torch.int8)
    sacts = acts.view(-1, S, Bs).permute(1, 0, 2).contiguous()
    c5 = cfg == "c5"
    F = int(L.wab_feature_dim(e0._h)) if c5 else 0
    keepalive = []

    def big(nbytes):
        if args.offset_kb < 0:
            return alloc(nbytes, dtype=torch.uint8, device=dev)
        x = alloc(nbytes + (2 << 30), dtype=torch.uint8, device=dev)
        keepalive.append(x)
        a = x.data_ptr()
        o = (-a) % (1 << 30) + args.offset_kb * 1024
        return x[o:o + nbytes]
    bufs = []
    for k in range(S):
        sc = alloc((3, T, Bs), dtype=torch.uint8, device=dev)
        pl = None if c5 else big(T * Bs * 3 * e0.W * e0.S).view(T, Bs, 3, e0.W, e0.S)
        bufs.append((_lib.WabObs(None if c5 else pl.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), sc[2].data_ptr()),
                     alloc((T, Bs), dtype=torch.float32, device=dev), alloc((T, Bs), dtype=torch.uint8, device=dev),
                     big(T * Bs * F * 4).view(torch.float32).view(T, Bs, F) if c5 else None,
                     alloc((T, Bs), dtype=torch.float32, device=dev), sc, pl))

    def roll(t, s, k=0):
        o, rd, dn, feats, ret, _, _ = bufs[k]
        if c5:
            _lib.check(L.wab_rollout_features(envs[k]._h, sacts[k].data_ptr() + t * Bs, T, ctypes.addressof(o),
                                              rd.data_ptr(), dn.data_ptr(), feats.data_ptr(), 0.99, None,
                                              ret.data_ptr(), s), "wab_rollout_features")
        else:
            _lib.check(L.wab_rollout(envs[k]._h, sacts[k].data_ptr() + t * Bs, T, ctypes.addressof(o), rd.data_ptr(),
                                     dn.data_ptr(), s), "wab_rollout")
    stream = torch.cuda.current_stream(dev)
    for t in range(0, W, T):
        for k in range(S):
            roll(t, ctypes.c_void_p(stream.cuda_stream), k)
    ms, n = bench.time_launches(lambda i, s, k=0: roll(W + i * T, s, k), NL, dev, stream, "graph", shards=S)
    c = [e.counters() for e in envs]
    big_ptrs = [(b[3] if c5 else b[6]).data_ptr() for b in bufs]
    print("  buffers at", ["%#x (mod 2MiB %#x, mod 1GiB %#x)" % (a, a % (1 << 21), a % (1 << 30)) for a in big_ptrs])
    print("%s prealloc %.1f GB zeros %d seed %d offset %d KiB: %.3f us per step (%d launches); resets per env-step %.4f"
          % (cfg, args.prealloc_gb, args.zeros, args.seed, args.offset_kb, ms * 1e3 / T, n,
             sum(x["resets"] for x in c) / max(1, sum(x["steps"] for x in c))))
    del keep


if __name__ == "__main__":
    main()
