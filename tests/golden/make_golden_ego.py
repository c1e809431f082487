"""Golden vectors for the egocentric observation variants, from the REAL reference.

Container-only (imports /root/reference through ref_harness).  Runs the unmodified
`WolvesAndBushesEnvEgoCentric` / `WolvesAndBushesEnvEgocentricJustBushes`
(wab_env.py:930-979) under the keyed RNG and records, per env and step, the 5 bush
proximities (`_get_bush_proximities`, wab_env.py:652-667: clip(max_distance - d, 0,
max_distance) with d the taxicab distance from the square each action would reach to the
nearest food>0 bush of the *whole generated world*, and max_distance when there is none),
plus food_turns / role / status, reward and done.

Protocol per env (autoreset, as make_golden.py): obs0 = constructor's reset; then
step(a[t]); on done the terminal obs is recorded, then reset() and the reset obs recorded.

Policies (chosen from the raw 7-tuple obs, `WolvesAndBushesEnv._get_obs`): random,
bush-seeking, and an explorer that walks straight for a while and then turns back, so that
bushes seen earlier but now outside the viewport decide the proximities.

Usage: python tests/golden/make_golden_ego.py [set ...]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as rh  # noqa: E402
from make_golden import choose_action  # noqa: E402

SEED = 0x5EED
EGO, JUST = "WolvesAndBushesEnvEgoCentric", "WolvesAndBushesEnvEgocentricJustBushes"
SETS = {
    # name: (options override, env ids, T, class)
    "ego_default": ({}, list(range(3000, 3024)), 120, EGO),
    "ego_wide31": ({"width": 31, "height": 31}, list(range(3100, 3108)), 90, EGO),
    # bush_power 400: ~1.5% of tiles hold food, so some worlds have no bush at all
    "ego_sparse": ({"bush_power": 400}, list(range(3200, 3216)), 100, EGO),
    # one berry per bush: every eaten bush empties (and leaves the proximity set)
    "ego_empty": ({"max_berries_per_bush": 1, "bush_power": 20}, list(range(3300, 3312)), 100, JUST),
    "ego_rect": ({"width": 13, "height": 9, "chance_wolf_on_square": 0.0}, list(range(3400, 3408)), 100,
                 JUST),
}


def explorer_action(rng, state, n_actions):
    """Walk in one direction for 6..20 steps, then back the other way for as long."""
    if state.get("left", 0) <= 0:
        if "dir" in state and not state.get("returning"):
            state["dir"] = (state["dir"] + 2) % 4
            state["returning"] = True
            state["left"] = state["len"]
        else:
            state["dir"] = int(rng.randint(4))
            state["len"] = state["left"] = int(rng.randint(6, 21))
            state["returning"] = False
    state["left"] -= 1
    if rng.random_sample() < 0.1:
        return int(rng.randint(n_actions))
    return state["dir"]


def run_set(name):
    opts, env_ids, T, cls = SETS[name]
    wab_env = rh.load_reference()
    full = dict(wab_env.default_game_options)
    full.update(opts)
    E = len(env_ids)
    out = {
        "reset0_prox": np.zeros((E, 5), np.uint8),
        "reset0_scalars": np.zeros((E, 3), np.uint8),
        "actions": np.zeros((T, E), np.int8),
        "prox": np.zeros((T, E, 5), np.uint8),
        "scalars": np.zeros((T, E, 3), np.uint8),
        "reward": np.zeros((T, E), np.float64),
        "done": np.zeros((T, E), np.bool_),
        "rprox": np.zeros((T, E, 5), np.uint8),
        "rscalars": np.zeros((T, E, 3), np.uint8),
        "pos": np.zeros((T, E, 2), np.int64),
    }
    base_obs = wab_env.WolvesAndBushesEnv._get_obs
    t0 = time.time()
    no_bush = 0

    def record(env, obs):
        prox = np.asarray(obs if cls == JUST else obs[0], dtype=np.int64)
        raw = base_obs(env)
        planes, f, r, s = rh.obs_arrays(raw)
        if cls == EGO:
            assert (int(obs[1]), int(obs[2]), int(obs[3])) == (f, r, s)
        return prox.astype(np.uint8), (f, r, s), planes

    for e, g in enumerate(env_ids):
        env = rh.make_env(SEED, g, opts, cls=cls)
        n_actions = env.action_space.n
        rng = np.random.RandomState(3000 + e)
        policy = e % 3
        pstate = {}
        prox, sc, planes = record(env, env._get_obs())
        out["reset0_prox"][e], out["reset0_scalars"][e] = prox, sc
        for t in range(T):
            if policy == 2:
                a = explorer_action(rng, pstate, n_actions)
            else:
                a = choose_action(rng, policy, planes, n_actions)
            out["actions"][t, e] = a
            obs, rew, done, _ = env.step(a)
            prox, sc, planes = record(env, obs)
            out["prox"][t, e], out["scalars"][t, e] = prox, sc
            out["reward"][t, e], out["done"][t, e] = float(rew), bool(done)
            o = env.ostriches.iloc[0]
            out["pos"][t, e] = (int(o.x), int(o.y))
            no_bush += int(env.bushes[env.bushes.food > 0].empty)
            if done:
                obs = env.reset()
                pstate = {}
                prox, sc, planes = record(env, obs)
                out["rprox"][t, e], out["rscalars"][t, e] = prox, sc
    meta = {
        "set": name, "seed": SEED, "env_ids": [int(g) for g in env_ids], "T": T, "class": cls,
        "protocol": "autoreset", "options": full, "generator": "tests/golden/make_golden_ego.py",
        "reference": "wab_env.py (johnmatthewtennant/wab-gym) under oracle/keyed_rng.py",
    }
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, "%s.npz" % name)
    np.savez_compressed(path, **out)
    print("%-11s E=%3d T=%3d dones=%4d no-bush-steps=%4d max|pos|=%3d  %.1fs -> %s" % (
        name, E, T, int(out["done"].sum()), no_bush, int(np.abs(out["pos"]).max()), time.time() - t0,
        os.path.basename(path)))


if __name__ == "__main__":
    for n in sys.argv[1:] or list(SETS):
        run_set(n)
