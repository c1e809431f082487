"""Golden vectors for the config-5 return scan: the reference's own `finish_episode`
(actor_critic.py:128-169) on reward sequences of episodes the reference env itself played.

Container-only (imports /root/reference through ref_harness; actor_critic.py needs torch,
which is here, and gym, which the harness shims).  Importing actor_critic builds its module
globals (actor_critic.py:42-105: the wrapped env, Policy, Adam); gym 0.17's Monitor is a
pass-through wrapper for that import (no files), and the env it builds draws from plain
numpy during the import only.  Then, per episode:

  * the rewards are the reference env's own step() rewards (Python doubles: e.g. 0.1 + -1 is
    -0.8999999999999999, not -0.9), from keyed-RNG episodes with random actions;
  * `model.rewards` gets them and `model.saved_actions` one (log_prob, value) pair per step
    (real tensors, so the loss, backward and Adam step of finish_episode run as written);
  * `actor_critic.torch` is wrapped so that `torch.tensor(returns)` (:145) records the exact
    double returns R = r + 0.99 R (:139-143), and `torch.tensor([R])` (:155) the normalised
    float32 returns (R - mean) / (std + eps) (:146).

Writes tests/golden/returns.npz: rewards (f64 exact, f32 as the device stores them), done
flags marking each episode's last step, returns (f64), normalised (f32).

Usage: python tests/golden/make_golden_returns.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as rh  # noqa: E402

SEED = 0x5EED
SETS = {
    # name: (options override, env ids)
    "default": ({}, list(range(3000, 3030))),
    "wolfy": ({"chance_wolf_on_square": 0.03, "wolf_chance_to_despawn": 0.2}, list(range(3100, 3110))),
    "eater": ({"bush_power": 20}, list(range(3200, 3210))),
}


def import_actor_critic():
    import gym

    wab_env = rh.load_reference()
    gym.wrappers.Monitor = lambda env, *a, **k: gym.Wrapper(env)  # pass-through (no video/stats files)
    keyed = wab_env.np
    wab_env.np = np  # the module-level env of actor_critic.py:42 draws from plain numpy
    np.random.seed(0)
    try:
        import actor_critic
    finally:
        wab_env.np = keyed
    return actor_critic


class _Recorder(types.SimpleNamespace):
    """actor_critic.torch stand-in: everything is torch, tensor() also records its data."""

    def __init__(self, torch):
        super().__init__()
        self._t = torch
        self.calls = []

    def __getattr__(self, name):
        return getattr(self._t, name)

    def tensor(self, data, *a, **k):
        self.calls.append(data)
        return self._t.tensor(data, *a, **k)


def episode_rewards(opts, env_id, rng):
    env = rh.make_env(SEED, env_id, opts)
    env.reset()
    rewards = []
    while True:
        _, r, done, _ = env.step(int(rng.randint(env.action_space.n)))
        rewards.append(r)
        if done:
            return rewards


def main():
    import torch

    ac = import_actor_critic()
    wab_env = rh.load_reference()
    rew64, done, ret64, norm32, set_ids = [], [], [], [], []
    for si, (name, (opts, ids)) in enumerate(SETS.items()):
        full = dict(wab_env.default_game_options)
        full.update(opts)
        rng = np.random.RandomState(5 + si)
        for g in ids:
            rewards = episode_rewards(full, g, rng)
            ac.model.rewards[:] = list(rewards)
            ac.model.saved_actions[:] = [
                ac.SavedAction(torch.log(torch.tensor(0.5, requires_grad=True)), torch.zeros(1, requires_grad=True))
                for _ in rewards]
            rec = _Recorder(torch)
            ac.torch = rec
            try:
                ac.finish_episode()
            finally:
                ac.torch = torch
            returns = [float(v) for v in rec.calls[0]]                 # torch.tensor(returns), :145
            normed = [float(c[0]) for c in rec.calls[1:1 + len(rewards)]]  # torch.tensor([R]), :155
            assert len(returns) == len(rewards) == len(normed)
            rew64 += [float(r) for r in rewards]
            done += [0] * (len(rewards) - 1) + [1]
            ret64 += returns
            norm32 += normed
            set_ids += [si] * len(rewards)
    out = {
        "rewards64": np.asarray(rew64, np.float64),
        "rewards32": np.asarray(rew64, np.float32),
        "done": np.asarray(done, np.uint8),
        "returns64": np.asarray(ret64, np.float64),
        "normalised32": np.asarray(norm32, np.float32),
        "set": np.asarray(set_ids, np.uint8),
        "gamma": np.float64(ac.gamma),
        "set_names": np.frombuffer(",".join(SETS).encode(), dtype=np.uint8),
    }
    np.savez_compressed(os.path.join(HERE, "returns.npz"), **out)
    print("returns.npz: %d episodes, %d steps, rewards %s" % (
        int(out["done"].sum()), len(rew64), sorted(set(np.round(out["rewards64"], 6)))))


if __name__ == "__main__":
    main()
