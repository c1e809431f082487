"""Replay backends for tests/golden_replay.py: the C oracle (CPU) and the HIP product (GPU)."""
from __future__ import annotations

import numpy as np

SEED = 0x5EED


class OracleBackend:
    def __init__(self, opts, base, n, autoreset, stride, seed=SEED):
        from oracle.oracle import OracleBatch

        self.o = OracleBatch(opts, n, seed, base, autoreset, stride)

    def reset(self):
        return tuple(x.copy() for x in self.o.reset())

    def step(self, a):
        p, f, r, s, rw, d = self.o.step(a)
        term = (self.o.t_planes.copy(), self.o.t_food_turns.copy(), self.o.t_role.copy(),
                self.o.t_status.copy())
        return p.copy(), f.copy(), r.copy(), s.copy(), rw.copy(), d.copy(), term

    def state(self):
        return self.o.state()


class GpuBackend:
    """The product path: BatchedWolvesAndBushesEnv -> ctypes -> libwab_hip.so (C-ABI)."""

    wolf_slots = 32

    def __init__(self, opts, base, n, autoreset, stride, seed=SEED):
        from wab_gym_amd.env import BatchedWolvesAndBushesEnv

        self.env = BatchedWolvesAndBushesEnv(opts, num_envs=n, seed=seed, device="cuda:0",
                                             env_id_base=base, autoreset=autoreset,
                                             return_terminal=True, plane_stride=stride,
                                             wolf_slots=self.wolf_slots)

    def _np(self, obs):
        return (self.env._obs["planes"].cpu().numpy(), obs[3].cpu().numpy(),
                obs[4].cpu().numpy(), obs[5].cpu().numpy())

    def reset(self):
        return self._np(self.env.reset())

    def step(self, a):
        import torch

        obs, rew, done, info = self.env.step(torch.as_tensor(np.asarray(a, np.int64)))
        planes, f, r, s = self._np(obs)
        t = self.env._term
        term = (t["planes"].cpu().numpy(), t["scalars"][0].cpu().numpy(),
                t["scalars"][1].cpu().numpy(), t["scalars"][2].cpu().numpy())
        return planes, f, r, s, rew.cpu().numpy(), done.cpu().numpy().astype(np.uint8), term

    def state(self):
        return self.env.state()


class GpuRolloutBackend:
    """The product's multi-step path: BatchedWolvesAndBushesEnv.rollout -> wab_rollout (one
    launch for the whole segment; no terminal observations, the bench's auto-reset path)."""

    wolf_slots = 32

    def __init__(self, opts, base, n, autoreset, stride, seed=SEED):
        from wab_gym_amd.env import BatchedWolvesAndBushesEnv

        self.env = BatchedWolvesAndBushesEnv(opts, num_envs=n, seed=seed, device="cuda:0",
                                             env_id_base=base, autoreset=autoreset,
                                             plane_stride=stride, wolf_slots=self.wolf_slots)

    def reset(self):
        obs = self.env.reset()
        return (self.env._obs["planes"].cpu().numpy(), obs[3].cpu().numpy(), obs[4].cpu().numpy(),
                obs[5].cpu().numpy())

    def rollout(self, actions):
        import torch

        planes, scal, rew, done = self.env.rollout(torch.as_tensor(np.asarray(actions, np.int64)))
        s = scal.cpu().numpy()
        return (planes.cpu().numpy(), s[:, 0], s[:, 1], s[:, 2], rew.cpu().numpy(), done.cpu().numpy())

    def state(self):
        return self.env.state()


class GpuPaddedRolloutBackend(GpuRolloutBackend):
    """GpuRolloutBackend over a batch padded to a multiple of 16 envs (extra envs get ids after
    the group's and action 0; their results are dropped), so that every step's plane slice is
    16-byte aligned and wab_rollout takes its one-launch path for the small and wide kernels:
    asserted from the handle's host tallies after every rollout."""

    def __init__(self, opts, base, n, autoreset, stride, seed=SEED):
        self.n = n
        super().__init__(opts, base, -(-n // 16) * 16, autoreset, stride, seed)
        self.one_launch = self.env.step_kernel in ("small", "wide")

    def reset(self):
        return tuple(x[:self.n] for x in super().reset())

    def rollout(self, actions):
        a = np.zeros((len(actions), self.env.num_envs), np.int64)
        a[:, :self.n] = actions
        before = self.env.counters()
        out = tuple(x[:, :self.n] for x in super().rollout(a))
        c = self.env.counters()
        launches = c["rollout_launches"] - before["rollout_launches"]
        per_step = c["rollout_step_calls"] - before["rollout_step_calls"]
        assert (launches, per_step) == ((1, 0) if self.one_launch else (0, 1)), (
            "rollout of %d envs (%s kernel) ran %d one-launch / %d per-step calls"
            % (self.env.num_envs, self.env.step_kernel, launches, per_step))
        return out

    def state(self):
        return {k: v[:self.n] for k, v in self.env.state().items()}
