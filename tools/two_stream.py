"""Experiment: the B = 65536 batch as S independent shards (env id bases 0, B/S, ...) stepped on
S streams, captured in one graph with a fork/join per step, vs one handle on one stream.
Prints us per step of the whole batch.  Usage (GPU box): python tools/two_stream.py [--shards 2]
"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--join-every", type=int, default=1, help="fork/join every n steps")
    ap.add_argument("--features", action="store_true",
                    help="C5's fused wab_step_features into a [32, n, F] buffer per shard instead of wab_step")
    args = ap.parse_args()
    import torch

    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    dev = torch.device("cuda", 0)
    S, B, K = args.shards, args.batch, args.steps
    n = B // S
    envs = [BatchedWolvesAndBushesEnv(None, num_envs=n, seed=0x5EED, device=dev, env_id_base=i * n,
                                      validate_actions=False) for i in range(S)]
    for e in envs:
        e.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    actions = torch.randint(0, 5, (K + 50, B), device=dev, generator=gen).to(torch.int8)
    L = _lib.load()
    main_s = torch.cuda.current_stream(dev)
    F = int(L.wab_feature_dim(envs[0]._h))
    feats = [torch.empty((32, n, F), dtype=torch.float32, device=dev) if args.features else None for _ in range(S)]
    fobs = []
    for e in envs:
        o = e._obs["struct"]
        fobs.append(_lib.WabObs(None, o.food_turns, o.role, o.status))
    streams = [torch.cuda.Stream(dev) for _ in range(S)]

    def step_all(t0, cnt):
        for t in range(t0, t0 + cnt, args.join_every):
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            for i, (e, st) in enumerate(zip(envs, streams)):
                st.wait_event(ev)
                for u in range(t, min(t + args.join_every, t0 + cnt)):
                    a = actions[u, i * n:(i + 1) * n]
                    if args.features:
                        _lib.check(L.wab_step_features(e._h, a.data_ptr(), ctypes.addressof(fobs[i]), e.reward.data_ptr(),
                                                       e.done.data_ptr(), feats[i][u % 32].data_ptr(),
                                                       ctypes.c_void_p(st.cuda_stream)), "wab_step_features")
                    else:
                        _lib.check(L.wab_step(e._h, a.data_ptr(), ctypes.addressof(e._obs["struct"]), e.reward.data_ptr(),
                                              e.done.data_ptr(), None, ctypes.c_void_p(st.cuda_stream)), "wab_step")
            for st in streams:
                torch.cuda.current_stream(dev).wait_stream(st)

    step_all(0, 50)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev)
    side.wait_stream(main_s)
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            step_all(50, K)
    main_s.wait_stream(side)
    torch.cuda.synchronize()
    for _ in range(2):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print("shards %d join_every %d: %.3f us per step of %d envs (%.2f G env-steps/s)"
              % (S, args.join_every, dt / K * 1e6, B, B * K / dt / 1e9), flush=True)


if __name__ == "__main__":
    main()
