"""Generate the committed golden vectors in tests/golden/*.npz from the REAL reference.

Container-only (needs /root/reference).  Runs the unmodified `wab_env.WolvesAndBushesEnv`
under the keyed RNG of `ref_harness.py` and records, per env and step, every output of the
reference surface (`step` -> obs 7-tuple, reward, done; `wab_env.py:250-342`) plus a few
hidden-state fields (raw food double, ostrich position, live wolf count) that pin the
restatement more tightly than the observation alone.

Protocol per env (matches the batched env's semantics):
  obs0 = reset()  (the constructor's reset, episode 0)
  for t in range(T):  obs, r, done = step(a[t]);  if done and protocol == "autoreset": reset()
"continue" sets never reset: they keep stepping after `done` (unguarded in the reference).

Actions are inputs: a per-env mix of random, bush-seeking and wolf-seeking policies
(seeded numpy RandomState), chosen so that eating, bush depletion, kills, starvation and
finishing at max_turns all occur.

Usage:  python tests/golden/make_golden.py [set ...]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as rh  # noqa: E402

SEED = 0x5EED

SETS = {
    # name: (options override, env ids, T, protocol)
    "default": ({}, list(range(40)) + [4095, 65535, 65536 * 7 + 12345, 2**40 + 3], 200, "autoreset"),
    "continue": ({}, list(range(100, 112)), 130, "continue"),
    "wide31": ({"width": 31, "height": 31}, list(range(200, 212)), 110, "autoreset"),
    "neither6": ({"lookout_only": False, "gatherer_only": False}, list(range(300, 312)), 120, "autoreset"),
    "gatherer": ({"gatherer_only": True, "lookout_only": False}, list(range(400, 410)), 100, "autoreset"),
    "static_god": ({"wolves_can_move": False, "god_mode": True, "chance_wolf_on_square": 0.02},
                   list(range(500, 510)), 100, "autoreset"),
    "nowolves": ({"wolves": False}, list(range(600, 606)), 90, "autoreset"),
    "rand_start": ({"starting_food": None, "starting_role": None}, list(range(700, 712)), 90, "autoreset"),
    "wolfy": ({"chance_wolf_on_square": 0.03, "wolf_chance_to_despawn": 0.2, "wolf_spawn_margin": 2},
              list(range(800, 812)), 100, "autoreset"),
    "restrict": ({"restrict_view": True, "lookout_only": False}, list(range(900, 910)), 100, "autoreset"),
    "rect9x13": ({"width": 13, "height": 11, "turns_to_fill_food": 4, "turns_to_empty_food": 30,
                  "max_turns": 60, "reward_for_eating": 0.25, "bush_power": 60},
                 list(range(1000, 1010)), 100, "autoreset"),
}


def choose_action(rng, policy, planes, n_actions):
    W, H = planes.shape[1:]
    cw, ch = W // 2, H // 2
    if policy == 0 or rng.random_sample() < 0.2:
        return int(rng.randint(n_actions))
    target = planes[1] if policy == 1 else planes[0]
    ii, jj = np.nonzero(target)
    if len(ii) == 0:
        return int(rng.randint(n_actions))
    d = np.abs(ii - cw) + np.abs(jj - ch)
    n = int(np.argmin(d))
    dx, dy = cw - ii[n], ch - jj[n]  # world offset of the target (grid axis 0 = ostrich_x - x)
    if dx == 0 and dy == 0:
        return 4 if n_actions == 5 or rng.random_sample() < 0.5 else 5
    if abs(dx) >= abs(dy):
        return 1 if dx > 0 else 3
    return 0 if dy > 0 else 2


def run_set(name):
    opts, env_ids, T, protocol = SETS[name]
    wab_env = rh.load_reference()
    full = dict(wab_env.default_game_options)
    full.update(opts)
    E = len(env_ids)
    W, H = full["width"], full["height"]
    nbits = 3 * W * H
    nbytes = (nbits + 7) // 8

    def pack(planes):
        return np.packbits(planes.reshape(-1))

    envs = [rh.make_env(SEED, g, opts) for g in env_ids]
    n_actions = envs[0].action_space.n
    out = {
        "reset0_bits": np.zeros((E, nbytes), np.uint8),
        "reset0_scalars": np.zeros((E, 3), np.uint8),
        "actions": np.zeros((T, E), np.int8),
        "bits": np.zeros((T, E, nbytes), np.uint8),
        "scalars": np.zeros((T, E, 3), np.uint8),
        "reward": np.zeros((T, E), np.float64),
        "done": np.zeros((T, E), np.bool_),
        "rbits": np.zeros((T, E, nbytes), np.uint8),
        "rscalars": np.zeros((T, E, 3), np.uint8),
        "food": np.zeros((T, E), np.float64),
        "pos": np.zeros((T, E, 2), np.int64),
        "n_wolves": np.zeros((T, E), np.int32),
        "view_mask": np.zeros((T, E, 11, 11), np.uint8),
    }
    t0 = time.time()
    for e, env in enumerate(envs):
        rng = np.random.RandomState(1000 + e)
        policy = e % 3
        obs = env._get_obs()  # the constructor's reset obs (episode 0)
        planes, f, r, s = rh.obs_arrays(obs)
        out["reset0_bits"][e] = pack(planes)
        out["reset0_scalars"][e] = (f, r, s)
        for t in range(T):
            a = choose_action(rng, policy, planes, n_actions)
            out["actions"][t, e] = a
            obs, rew, done, _ = env.step(a)
            planes, f, r, s = rh.obs_arrays(obs)
            out["bits"][t, e] = pack(planes)
            out["scalars"][t, e] = (f, r, s)
            out["reward"][t, e] = float(rew)
            out["done"][t, e] = bool(done)
            out["view_mask"][t, e] = np.asarray(obs[6], dtype=np.uint8)
            o = env.ostriches.iloc[0]
            out["food"][t, e] = float(o.food)
            out["pos"][t, e] = (int(o.x), int(o.y))
            out["n_wolves"][t, e] = len(env.wolves)
            if done and protocol == "autoreset":
                obs = env.reset()
                planes, f, r, s = rh.obs_arrays(obs)
                out["rbits"][t, e] = pack(planes)
                out["rscalars"][t, e] = (f, r, s)
    meta = {
        "set": name, "seed": SEED, "env_ids": [int(g) for g in env_ids], "T": T,
        "protocol": protocol, "options": full, "n_actions": int(n_actions),
        "width": W, "height": H, "generator": "tests/golden/make_golden.py",
        "reference": "wab_env.py (johnmatthewtennant/wab-gym) under oracle/keyed_rng.py",
    }
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, "%s.npz" % name)
    np.savez_compressed(path, **out)
    print("%-11s E=%3d T=%3d dones=%4d eats~%5d maxwolves=%d  %.1fs -> %s" % (
        name, E, T, int(out["done"].sum()),
        int(np.isclose(out["reward"] - np.round(out["reward"]), full["reward_for_eating"]).sum()),
        int(out["n_wolves"].max()), time.time() - t0, os.path.basename(path)))


if __name__ == "__main__":
    names = sys.argv[1:] or list(SETS)
    for n in names:
        run_set(n)
