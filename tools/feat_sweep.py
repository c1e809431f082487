"""Featurizer (wab_featurize) launch time against batch size: separates the fixed latency of
a launch from its store throughput.  Usage (GPU box): python tools/feat_sweep.py"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from wab_gym_amd import _lib
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv

    L = _lib.load()
    out = []
    for B in (4096, 16384, 65536, 262144):
        env = BatchedWolvesAndBushesEnv(None, num_envs=B, device="cuda:0", validate_actions=False)
        env.reset()
        F = int(L.wab_feature_dim(env._h))
        feats = torch.empty((B, F), dtype=torch.float32, device="cuda:0")
        a = torch.randint(0, 5, (B,), device="cuda:0").to(torch.int8)
        for _ in range(20):
            env.step(a)
        s = torch.cuda.current_stream()
        sp = ctypes.c_void_p(s.cuda_stream)
        st = ctypes.addressof(env._obs["struct"])
        for _ in range(10):
            L.wab_featurize(env._h, st, None, feats.data_ptr(), sp)
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            L.wab_featurize(env._h, st, None, feats.data_ptr(), sp)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        out.append({"B": B, "us": round(us, 2), "write_GBs": round(B * F * 4 / us / 1e3, 1)})
        env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
