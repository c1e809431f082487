"""Debug: run one option set on the GPU and the oracle in lockstep, print the first env whose
obs differs (per plane cell diffs) with both states before and after."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle.oracle import OracleBatch  # noqa: E402
from wab_gym_amd.env import BatchedWolvesAndBushesEnv  # noqa: E402

opts = json.loads(sys.argv[1])
stride, slots, n, T = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
env = BatchedWolvesAndBushesEnv(opts, num_envs=n, seed=0x5EED, device="cuda:0", env_id_base=5,
                                return_terminal=True, plane_stride=stride, wolf_slots=slots)
orc = OracleBatch(opts, n, 0x5EED, 5, True, stride)
env.reset()
orc.reset()
print("kernel", env.step_kernel)
rng = np.random.RandomState(0)
prev_g, prev_o = env.state(), orc.state()
for t in range(T):
    a = rng.randint(env.n_actions, size=n)
    env.step(torch.as_tensor(a))
    orc.step(a, nthreads=16)
    gp = env._obs["planes"].cpu().numpy()
    op = orc.planes
    sg, so = env.state(), orc.state()
    bad = np.nonzero((gp != op).reshape(n, -1).any(1))[0]
    if len(bad):
        e = bad[0]
        print("t", t, "bad envs", bad[:20], "action", a[e])
        for k in range(3):
            d = np.argwhere(gp[e, k] != op[e, k])
            if len(d):
                print(" plane", k, "cells", d[:20].tolist(), "gpu", gp[e, k][tuple(d.T)][:20], "orc", op[e, k][tuple(d.T)][:20])
        for name, st in (("gpu prev", prev_g), ("orc prev", prev_o), ("gpu", sg), ("orc", so)):
            print(" ", name, {k: st[k][e] for k in st})
        print(" done", env.done[e].item(), orc.done[e], "status", orc.status[e])
        print(" counters", env.counters())
        break
    prev_g, prev_o = sg, so
else:
    print("no diff", env.counters())
