"""Python-level env.step() rate at B = 65536 (drop-in surface, one call per step, device
actions) for each validate_actions mode: True (the default: checked by the kernel, raised at
the next synchronising call), "sync" (one blocking check per step) and False."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from wab_gym_amd.env import BatchedWolvesAndBushesEnv
    from wab_gym_amd.wrappers import PragmaticObsWrapper

    B, K = 65536, 300
    acts = torch.randint(0, 5, (K, B), device="cuda:0", dtype=torch.int8)
    for validate in (True, "sync", False):
        env = BatchedWolvesAndBushesEnv(num_envs=B, device="cuda:0", validate_actions=validate)
        env.reset()
        for k in range(20):
            env.step(acts[k])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            env.step(acts[k])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        env.check()
        print("env.step validate_actions=%s: %.1f us/step, %.2f G env-steps/s" % (validate, dt * 1e6, B / dt / 1e9))
    w = PragmaticObsWrapper(BatchedWolvesAndBushesEnv(num_envs=B, device="cuda:0"))
    w.reset()
    for k in range(20):
        w.step(acts[k])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        w.step(acts[k])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print("PragmaticObsWrapper.step (fused, planes stored): %.1f us/step, %.2f G env-steps/s" % (dt * 1e6, B / dt / 1e9))


if __name__ == "__main__":
    main()
