"""Monitor-style episode statistics for a batched env.

The reference wraps its env in gym 0.17's `gym.wrappers.Monitor` (actor_critic.py:46,
wab_env.py:1013), whose stats recorder sums each episode's rewards as Python floats in step
order (starting from the int 0) and counts its steps, and on close writes
`openaigym.episode_batch.<infix>.stats.json` with `initial_reset_timestamp`, `timestamps`,
`episode_lengths`, `episode_rewards` and `episode_types`.  gym is not installed here, so the
file layout is a restatement of gym 0.17's stats recorder (parity unpinned); the episode sums
themselves are pinned bit for bit against sums of the reference's own double rewards in the
golden vectors (tests/test_monitor.py).  Videos are not recorded.

The device reward is the reference's double reward rounded to float32 (include/wab.h).  Each
step's double is recovered exactly from the few values a step can produce, `r_x` or
`r_eat + r_x` for r_x in (per turn, finishing, starving, killed) (wab_env.py:299-340), then
summed in float64 on device.  Finished episodes are gathered every `flush_every` steps (one
host synchronisation), so the per-step path stays asynchronous.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

_REWARD_KEYS = ("reward_per_turn", "reward_for_finishing", "reward_for_starving", "reward_for_being_killed")


def reward_table(game_options):
    """[(float32 value, exact double)] of every reward a step can return (wab_env.py:299-340):
    `0 + r_x` without an eat, `0 + r_eat + r_x` with one."""
    r_eat = game_options["reward_for_eating"]
    pairs = {}
    for k in _REWARD_KEYS:
        rx = game_options[k]
        for d in (0 + rx, 0 + r_eat + rx):
            d = float(d)
            f = float(np.float32(d))
            if f in pairs and pairs[f] != d:
                raise ValueError("rewards %r and %r round to the same float32: the double sum is "
                                 "not recoverable from the device reward" % (pairs[f], d))
            pairs[f] = d
    return sorted(pairs.items())


class EpisodeStats:
    """Per-env episode return (float64) and length on device; finished episodes are gathered
    into host lists in (step, env) order by flush()."""

    def __init__(self, game_options, num_envs, device, flush_every=32):
        import torch

        self._torch = torch
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.flush_every = int(flush_every)
        tab = reward_table(game_options)
        self._f32 = torch.tensor([f for f, _ in tab], dtype=torch.float32, device=self.device)
        self._f64 = torch.tensor([d for _, d in tab], dtype=torch.float64, device=self.device)
        B, K = self.num_envs, self.flush_every
        self.ret = torch.zeros(B, dtype=torch.float64, device=self.device)
        self.length = torch.zeros(B, dtype=torch.int64, device=self.device)
        self._buf_ret = torch.zeros((K, B), dtype=torch.float64, device=self.device)
        self._buf_len = torch.zeros((K, B), dtype=torch.int64, device=self.device)
        self._times = []
        self.episode_rewards, self.episode_lengths, self.episode_envs = [], [], []
        self.timestamps, self.episode_types = [], []
        self.total_steps = 0

    def restart(self, mask=None):
        """Start new episodes (all envs, or those with mask[i]); unfinished ones are dropped."""
        if mask is None:
            self.ret.zero_()
            self.length.zero_()
        else:
            m = self._torch.as_tensor(mask, device=self.device).bool()
            self.ret.masked_fill_(m, 0.0)
            self.length.masked_fill_(m, 0)

    def decode(self, reward):
        """float32 device rewards -> the reference's doubles."""
        r = reward.to(self._torch.float32)
        hit = r.unsqueeze(1) == self._f32.unsqueeze(0)  # [B, n_values]
        exact = (hit.to(self._torch.float64) * self._f64.unsqueeze(0)).sum(1)
        return self._torch.where(hit.any(1), exact, r.to(self._torch.float64))

    def update(self, reward, done):
        """One step of every env: add the step's reward, count it, close the done episodes."""
        t = self._torch
        d = t.as_tensor(done, device=self.device).bool()
        self.ret += self.decode(t.as_tensor(reward, device=self.device))
        self.length += 1
        k = len(self._times)
        self._buf_ret[k].copy_(self.ret)
        self._buf_len[k].copy_(t.where(d, self.length, t.zeros_like(self.length)))
        self._times.append(time.time())
        self.ret.masked_fill_(d, 0.0)
        self.length.masked_fill_(d, 0)
        self.total_steps += self.num_envs
        if len(self._times) == self.flush_every:
            self.flush()

    def flush(self):
        """Gather the episodes finished since the last flush (synchronises)."""
        k = len(self._times)
        if k == 0:
            return
        lens = self._buf_len[:k].cpu().numpy()
        rets = self._buf_ret[:k].cpu().numpy()
        steps, envs = np.nonzero(lens)
        self.episode_rewards.extend(float(x) for x in rets[steps, envs])
        self.episode_lengths.extend(int(x) for x in lens[steps, envs])
        self.episode_envs.extend(int(x) for x in envs)
        self.timestamps.extend(self._times[s] for s in steps)
        self.episode_types.extend("t" for _ in steps)
        self._times = []


class EpisodeMonitor:
    """`gym.wrappers.Monitor(env, directory, force)` for a batched env: episode statistics only
    (no video).  Attributes of the wrapped env pass through."""

    def __init__(self, env, directory=None, force=False, flush_every=32, monitor_id=0):
        self.env = env
        self.stats = EpisodeStats(env.game_options, env.num_envs, env.device, flush_every)
        self.directory = directory
        self.initial_reset_timestamp = None
        self._infix = "%d.%d" % (monitor_id, os.getpid())
        if directory is not None:
            os.makedirs(directory, exist_ok=True)
            if force:
                for f in os.listdir(directory):
                    if f.startswith("openaigym."):
                        os.remove(os.path.join(directory, f))

    def __getattr__(self, name):
        return getattr(self.env, name)

    def reset(self, mask=None):
        obs = self.env.reset(mask)
        if self.initial_reset_timestamp is None:
            self.initial_reset_timestamp = time.time()
        self.stats.restart(mask)
        return obs

    def step(self, actions):
        obs, reward, done, info = self.env.step(actions)
        self.stats.update(reward, done)
        return obs, reward, done, info

    def get_episode_rewards(self):
        self.stats.flush()
        return list(self.stats.episode_rewards)

    def get_episode_lengths(self):
        self.stats.flush()
        return list(self.stats.episode_lengths)

    def get_total_steps(self):
        return self.stats.total_steps

    def write_stats(self):
        """The stats file of gym 0.17's stats recorder (+ a manifest naming it)."""
        self.stats.flush()
        if self.directory is None:
            return None
        s = self.stats
        path = os.path.join(self.directory, "openaigym.episode_batch.%s.stats.json" % self._infix)
        with open(path, "w") as f:
            json.dump({"initial_reset_timestamp": self.initial_reset_timestamp,
                       "timestamps": s.timestamps, "episode_lengths": s.episode_lengths,
                       "episode_rewards": s.episode_rewards, "episode_types": s.episode_types}, f)
        spec = getattr(self.env, "spec", None)
        with open(os.path.join(self.directory, "openaigym.manifest.%s.manifest.json" % self._infix), "w") as f:
            json.dump({"stats": os.path.basename(path), "videos": [],
                       "env_info": {"env_id": getattr(spec, "id", None), "gym_version": "0.17.2 (restated)"}}, f)
        return path

    def close(self):
        path = self.write_stats()
        self.env.close()
        return path
