"""The headline rollout as S shards of B / S envs on S streams (each shard's T-step wab_rollout
launches in order on its own stream, the shards independent), against one handle of B envs:
does one shard's launch tail overlap another's work?  Prints us per batched step for both."""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--launches", type=int, default=48)
    ap.add_argument("--config", default="default", help="bench.py config: default, wide31 or c5")
    ap.add_argument("--stagger", action="store_true",
                    help="odd shards start (and end) with a T/2-step launch, so the shards' launch ends alternate")
    args = ap.parse_args()
    import torch

    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    L = _lib.load()
    dev = torch.device("cuda:0")
    B, T, S, K = args.batch, args.T, args.shards, args.launches

    import bench

    opts, stride, slots, _ = bench.CONFIGS[args.config]
    c5 = args.config == "c5"

    def setup(n, base):
        env = BatchedWolvesAndBushesEnv(opts, num_envs=n, seed=0x5EED, device=dev, env_id_base=base,
                                        validate_actions=False, wolf_slots=slots, plane_stride=stride)
        env.reset()
        acts = torch.randint(0, env.n_actions, (T, n), device=dev).to(torch.int8)
        pl = None if c5 else torch.empty((T, n, 3, env.W, env.S), dtype=torch.uint8, device=dev)
        sc = torch.empty((3, T, n), dtype=torch.uint8, device=dev)
        rw = torch.empty((T, n), dtype=torch.float32, device=dev)
        dn = torch.empty((T, n), dtype=torch.uint8, device=dev)
        o = _lib.WabObs(None if c5 else pl.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), sc[2].data_ptr())
        extra = None
        if c5:
            F = int(L.wab_feature_dim(env._h))
            extra = (torch.empty((T, n, F), dtype=torch.float32, device=dev),
                     torch.empty((T, n), dtype=torch.float32, device=dev))
        return env, acts, (pl, extra), sc, rw, dn, o

    def launch_one(shard, st, n):
        env, acts, pl, sc, rw, dn, o = shard
        if c5:
            f, ret = pl[1]
            _lib.check(L.wab_rollout_features(env._h, acts.data_ptr(), n, ctypes.addressof(o), rw.data_ptr(),
                                              dn.data_ptr(), f.data_ptr(), 0.99, None, ret.data_ptr(),
                                              ctypes.c_void_p(st.cuda_stream)), "wab_rollout_features")
        else:
            _lib.check(L.wab_rollout(env._h, acts.data_ptr(), n, ctypes.addressof(o), rw.data_ptr(),
                                     dn.data_ptr(), ctypes.c_void_p(st.cuda_stream)), "wab_rollout")

    def launch_all(shards, streams, k):
        for sh, st in zip(shards, streams):
            launch_one(sh, st, T)

    def run(shards, streams):
        for it in range(2):  # warm-up, then timed
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K if it else 4):
                launch_all(shards, streams, k)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        return el / (K * T) * 1e6

    def run_graph(shards):
        # one graph: the shards' chains of K launches each, forked from the capture stream and
        # joined at its end; replayed and timed with events
        main = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(main):
            with torch.cuda.graph(g, stream=main):
                cap = torch.cuda.current_stream(dev)
                subs = [cap] + [torch.cuda.Stream(dev) for _ in shards[1:]]
                for st in subs[1:]:
                    st.wait_stream(cap)
                if args.stagger and len(shards) > 1:
                    for k in range(K + 1):
                        for j, (sh, st) in enumerate(zip(shards, subs)):
                            if j % 2 == 0:
                                if k < K:
                                    launch_one(sh, st, T)
                            else:
                                launch_one(sh, st, T // 2 if k in (0, K) else T)
                else:
                    for k in range(K):
                        launch_all(shards, subs, k)
                for st in subs[1:]:
                    cap.wait_stream(st)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st = torch.cuda.current_stream(dev)
        e0.record(st)
        for _ in range(3):
            g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (3 * K * T)

    one = [setup(B, 0)]
    us1 = run(one, [torch.cuda.current_stream(dev)])
    g1 = run_graph(one)
    del one
    torch.cuda.empty_cache()
    sh = [setup(B // S, k * (B // S)) for k in range(S)]
    sts = [torch.cuda.Stream(dev) for _ in range(S)]
    usS = run(sh, sts)
    gS = run_graph(sh)
    print("%s%s B=%d T=%d: one handle %.3f us per step (graph %.3f); %d shards on %d streams %.3f (graph %.3f)"
          % (args.config, " (staggered)" if args.stagger else "", B, T, us1, g1, S, S, usS, gS))


if __name__ == "__main__":
    main()
