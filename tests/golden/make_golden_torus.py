"""Generate the committed torus-world golden vectors tests/golden/torus_*.npz from the REAL
Environment 2.0 reference (container-only: needs /root/reference).

Drives the unmodified `WAB_Environment2` / `World` (`Environment 2.0/WAB_Environment2.py:53-134`,
`World.py:93-395`) through its own surface, under the keyed `random` of `torus_harness.py`:

    env = WAB_Environment2(W, H, options)
    env.create_ostriches(n_o); env.create_wolves(n_w); env.create_bushes(n_b)   (random positions)
    env.reset_environment()
    per turn:  for entity i in id order:  obs = env.get_obs(i);  a = policy(obs);
                                          reward, done = env.take_action(i, a)
               "autoreset" sets: reset_environment() after a turn in which every ostrich is done
               or the world's turn count reached options["max_turns"] (the batched surface's
               episode rule; the reference itself never resets on its own)

Recorded per turn and world: every entity's get_obs() (visible-objects frame + internal obs)
encoded as the fixed-size record of include/wab_torus.h (`torus_harness.encode_obs`), the
(reward, done) take_action returned, the actions, whether the world was reset after the turn,
and hidden state after the turn: the frame's X/Y, the entity objects' x/y, food, the Visible
column and the ostriches' status.

Actions are inputs: ostriches walk to the nearest visible bush or at random (role actions 4/5
included), wolves chase the nearest visible ostrich or walk at random, bushes send 0; a few
actions outside every branch of the act functions (World.py:25-43, 61-73) are mixed in.

Usage:  python tests/golden/make_golden_torus.py [set ...]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import torus_harness as th  # noqa: E402

SEED = 0x5EED

# the policy's knobs: an ostrich seeks the nearest visible bush when u < ostrich_bush, a wolf
# chases the nearest visible ostrich with probability wolf_chase
POLICY = {"ostrich_bush": 0.6, "wolf_chase": 0.55}
# the hunt worlds of torus_c3: wolves always chase, the ostrich walks at random (kills, and
# the kill-triggered early resets of the benched 1/8/16 instance)
HUNT = {"ostrich_bush": 0.0, "wolf_chase": 1.0}


SETS = {
    # name: (W, H, (n_ostriches, n_wolves, n_bushes), option overrides, world ids, turns, protocol)
    # BASELINE config 3's literal reading: 32x32 torus, 1 ostrich, 8 wolves, 16 bushes
    # (+ six hunt worlds 400-405, policy HUNT: kills and kill-triggered early resets at 1/8/16)
    "torus_c3": (32, 32, (1, 8, 16), {}, list(range(8)) + [65535, 2**33 + 7] + list(range(400, 406)), 170,
                 "autoreset"),
    # several ostriches (eat order, the Visible-label quirk of World.py:115), a rectangular
    # world whose lookout radius reaches past the middle (both wrap branches), bushes that run
    # dry through take_food's second branch (12 -> 7 -> 2 -> 0)
    "torus_multi": (12, 10, (3, 4, 9), {"food_per_bush": 12, "lookout_view_radius": 7,
                                        "gatherer_view_radius": 3, "wolf_view_radius": 4,
                                        "max_turns": 50},
                    list(range(100, 106)), 130, "autoreset"),
    # a crowded 6x6 world: ties on every tile, a lookout radius larger than the world
    # (only the `if` branch of World.py:255/276 runs), lookouts from the start
    "torus_tiny": (6, 6, (2, 6, 10), {"lookout_view_radius": 9, "gatherer_view_radius": 1,
                                      "wolf_view_radius": 2, "starting_role": 0, "max_turns": 40,
                                      "food_per_bush": 7, "food_given_per_turn": 3,
                                      "wolf_starting_food": 6, "wolf_food_for_eating_ostrich": 4,
                                      "ostrich_starting_food": 2.5},
                   list(range(200, 206)), 120, "autoreset"),
    # no resets: the world runs on after its ostrich is dead
    "torus_continue": (16, 16, (1, 3, 5), {}, list(range(300, 304)), 140, "continue"),
    # caller-chosen positions: create_*(n, spawn_positions) and each entity's
    # reset(new_x, new_y) (WAB_Environment2.py:61-110, WAB_Environment2_Single.py:36-41) at turns
    # 0, 30 and 61, a quarter of them negative (the random position), some on the far edge;
    # the World_tests.py world size
    "torus_placed": (20, 20, (2, 3, 4), {"lookout_view_radius": 10, "gatherer_view_radius": 8,
                                         "wolf_view_radius": 6, "max_turns": 40},
                     list(range(500, 504)), 90, "autoreset"),
}
# per-set extras: the hunt worlds' policy; the placed set's explicit resets (turn -> positions)
POLICIES = {"torus_c3": {g: HUNT for g in range(400, 406)}}
PLACED_RESETS = {"torus_placed": (0, 30, 61)}


def placed_positions(e, W, H, N, k):
    """The placed set's positions of world index e: k = -1 create (tiles of the world), k >= 0
    the k-th explicit reset ((-1, -1) = random, x = W or y = H, or a tile)."""
    rng = np.random.RandomState(7000 + 97 * e + k)
    if k < 0:
        return np.stack([rng.randint(W, size=N), rng.randint(H, size=N)], -1).astype(np.int32)
    out = np.zeros((N, 2), np.int32)
    for i in range(N):
        u = rng.random_sample()
        if u < 0.25:
            out[i] = (-1, -1) if rng.random_sample() < 0.5 else (-1 - rng.randint(3), rng.randint(H))
        elif u < 0.4:  # on the far edges, x = W or y = H (as randint(0, W) draws them too)
            out[i] = (W, rng.randint(H + 1)) if rng.random_sample() < 0.5 else (rng.randint(W + 1), H)
        else:
            out[i] = (rng.randint(W + 1), rng.randint(H + 1))
    return out


def reset_at(env, pos):
    """reset_environment (WAB_Environment2.py:113-118) with each entity's reset(new_x, new_y)
    (WAB_Environment2_Single.py:36-41) instead of its argument-less call: the same body, driving
    the unmodified modules (the keyed episode counter as KeyedEnv2.reset_environment keeps it)."""
    env._world._wab_episode += 1
    for single, (x, y) in zip(env._environments, pos):
        single.reset(int(x), int(y))
    env.num_entities_acted_this_turn = 0
    env._world.reset_world()

JUNK = [-128, -1, 6, 7, 17, 127]


def _nearest(rec, off, types, want, rng):
    vis = int(np.frombuffer(rec[off["visible"]:off["visible"] + 4].tobytes(), np.uint32)[0])
    best = None
    for j, t in enumerate(types):
        if t == want and vis >> j & 1:
            dx = int(np.int8(rec[off["delta"] + 2 * j]))
            dy = int(np.int8(rec[off["delta"] + 2 * j + 1]))
            d = abs(dx) + abs(dy)
            if best is None or d < best[0]:
                best = (d, dx, dy)
    return best


def choose_action(rng, kind, rec, off, types, policy=POLICY):
    if rng.random_sample() < 0.03:
        return int(JUNK[rng.randint(len(JUNK))])
    if kind == "Bush":
        return 0
    if kind == "Ostrich":
        u = rng.random_sample()
        if u < 0.06:
            return int(4 + rng.randint(2))
        tgt = _nearest(rec, off, types, "Bush", rng) if u < policy["ostrich_bush"] else None
        if tgt is None:
            return int(rng.randint(6))
    else:
        tgt = _nearest(rec, off, types, "Ostrich", rng) if rng.random_sample() < policy["wolf_chase"] else None
        if tgt is None:
            return int(rng.randint(5))
    _, dx, dy = tgt
    if dx == 0 and dy == 0:
        return 4 if kind == "Wolf" else int(rng.randint(6))
    if abs(dx) >= abs(dy):
        return 1 if dx > 0 else 3
    return 0 if dy > 0 else 2


def run_set(name):
    W, H, (no, nw, nb), opts, world_ids, T, protocol = SETS[name]
    N = no + nw + nb
    types = ["Ostrich"] * no + ["Wolf"] * nw + ["Bush"] * nb
    R, off = th.record_layout(N, nb)
    E = len(world_ids)
    m = th.load_reference()
    full = dict(m["WAB_Environment2"].default_game_options)
    full.update(opts)
    out = {
        "actions": np.zeros((T, E, N), np.int8),
        "records": np.zeros((T, E, N, R), np.uint8),
        "reward": np.zeros((T, E, N), np.float64),
        "done": np.zeros((T, E, N), np.bool_),
        "world_reset": np.zeros((T, E), np.bool_),
        "df_xy": np.zeros((T, E, N, 2), np.int32),
        "obj_xy": np.zeros((T, E, N, 2), np.int32),
        "food": np.zeros((T, E, N), np.float64),
        "visible": np.zeros((T, E, N), np.bool_),
        "status": np.zeros((T, E, max(no, 1)), np.uint8),
        "create_df_xy": np.zeros((E, N, 2), np.int32),
        "reset0_obj_xy": np.zeros((E, N, 2), np.int32),
    }
    placed = PLACED_RESETS.get(name)
    if placed:
        out["create_pos"] = np.zeros((E, N, 2), np.int32)
        out["reset_pos"] = np.zeros((len(placed), E, N, 2), np.int32)
    t0 = time.time()
    kills = eats = resets = 0
    for e, g in enumerate(world_ids):
        rng = np.random.RandomState(5000 + e)
        policy = POLICIES.get(name, {}).get(g, POLICY)
        env = th.make_env(SEED, g, W, H, opts)
        if placed:
            cp = placed_positions(e, W, H, N, -1)
            out["create_pos"][e] = cp
            env.create_ostriches(no, [tuple(map(int, p)) for p in cp[:no]])
            env.create_wolves(nw, [tuple(map(int, p)) for p in cp[no:no + nw]])
            env.create_bushes(nb, [tuple(map(int, p)) for p in cp[no + nw:]])
        else:
            env.create_ostriches(no)
            env.create_wolves(nw)
            env.create_bushes(nb)
        ents = env._world._entities
        out["create_df_xy"][e] = ents[["X", "Y"]].to_numpy(np.int64)
        if placed:
            out["reset_pos"][0, e] = placed_positions(e, W, H, N, 0)
            reset_at(env, out["reset_pos"][0, e])
        else:
            env.reset_environment()
        out["reset0_obj_xy"][e] = [(o.x, o.y) for o in ents["Entity_Object"]]
        for t in range(T):
            if placed and t in placed[1:]:
                k = placed.index(t)
                out["reset_pos"][k, e] = placed_positions(e, W, H, N, k)
                reset_at(env, out["reset_pos"][k, e])
            for i in range(N):
                rec = out["records"][t, e, i]
                th.encode_obs(env.get_obs(i), i, types, nb, rec)
                a = choose_action(rng, types[i], rec, off, types, policy)
                out["actions"][t, e, i] = a
                r, d = env.take_action(i, a)
                out["reward"][t, e, i] = float(r)
                out["done"][t, e, i] = bool(d)
            objs = list(ents["Entity_Object"])
            st = [o.get_status() for o in objs[:no]]
            if protocol == "autoreset" and ((no > 0 and all(s != 0 for s in st)) or
                                            env._world._current_turn >= full["max_turns"]):
                env.reset_environment()
                out["world_reset"][t, e] = True
                resets += 1
            out["df_xy"][t, e] = ents[["X", "Y"]].to_numpy(np.int64)
            out["obj_xy"][t, e] = [(o.x, o.y) for o in objs]
            out["food"][t, e] = [float(o.food) for o in objs]
            out["visible"][t, e] = ents["Visible"].to_numpy(bool)
            out["status"][t, e, :no] = [o.get_status() for o in objs[:no]]
        kills += int((out["reward"][:, e, :no] == 0).sum())
        eats += int(np.diff(out["food"][:, e, :no], axis=0).clip(min=0).astype(bool).sum())
    meta = {"set": name, "seed": SEED, "world_ids": [int(g) for g in world_ids], "T": T,
            "protocol": protocol, "width": W, "height": H, "num_ostriches": no, "num_wolves": nw,
            "num_bushes": nb, "record_size": R, "options": full,
            "hunt_worlds": sorted(int(g) for g in POLICIES.get(name, {})),
            "placed_resets": list(placed) if placed else [],
            "generator": "tests/golden/make_golden_torus.py",
            "reference": "Environment 2.0/WAB_Environment2.py + World.py (johnmatthewtennant/wab-gym) "
                         "under the keyed random of tests/golden/torus_harness.py",
            "pandas": th.pd.__version__}
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    path = os.path.join(HERE, "%s.npz" % name)
    np.savez_compressed(path, **out)
    print("%-15s E=%2d T=%3d N=%2d R=%3d resets=%3d dead-ostrich-turns=%4d eats=%4d  %.1fs -> %s" % (
        name, E, T, N, R, resets, kills, eats, time.time() - t0, os.path.basename(path)))


if __name__ == "__main__":
    for n in sys.argv[1:] or list(SETS):
        run_set(n)
