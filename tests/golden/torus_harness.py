"""Run the *real* Environment 2.0 reference (`WAB_Environment2` / `World`) under a keyed RNG.

TEST INFRASTRUCTURE, container-only: used by `make_golden_torus.py` to produce the committed
fixtures `tests/golden/torus_*.npz`.  Nothing here runs on the GPU box.

The reference modules (`Environment 2.0/World.py`, `WAB_Environment2.py`,
`WAB_Environment2_Single.py`, `Entity.py`, `Wolf.py`, `Bush.py`, `Ostrich.py`) are imported
UNMODIFIED, with two stand-ins:
  1. `shims/gym` (gym is not installed; the modules only subclass `gym.Env`).
  2. each module's global `random` is replaced by `KeyedRandom`, whose `randint(a, b)` is a
     pure function of what the draw is about (oracle/keyed_rng.py, sites 7-10), found from
     the caller's frame:
       create_ostriches/_wolves/_bushes list comprehension (WAB_Environment2.py:64-106)
           site 7, episode 0, tile (entity id, axis)
       WAB_Environment2_Single._get_random_spawn_indices (WAB_Environment2_Single.py:43-48)
           site 8, episode = reset_environment() calls so far, tile (entity id, axis)
       default_game_update, wolf branch (World.py:112)       site 9 ... kill: site 10,
       default_game_update, ostrich branch (World.py:125)    turn = World._current_turn,
                                                              tile (acting entity id, 0)
     The axis (x or y) is read from the source line of the call (`get_width` / `get_height`).

Nothing else is patched: the quirks of the code as it runs on this container's pandas
(2.3.3) stay in the fixtures — the chained assignments `self._entities.iloc[j]["Visible"] =
False` (World.py:131) and `self._entities.iloc[i]["X"] = ...` (World.py:355-356) are no-ops
(a mixed-dtype row is a copy), so bushes never turn invisible and the frame's X/Y keep the
pre-reset positions until each entity acts; `self._entities.loc[j, "Visible"] = False`
(World.py:115) hides the ostrich whose LABEL is the tie-break index j, not the one killed.
"""
from __future__ import annotations

import linecache
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = os.environ.get("WAB_REFERENCE", "/root/reference")
ENV2_DIR = os.path.join(REFERENCE, "Environment 2.0")

sys.path.insert(0, os.path.join(HERE, "shims"))
sys.path.insert(0, REPO)

import pandas as pd  # noqa: E402

from oracle import keyed_rng as kr  # noqa: E402

warnings.filterwarnings("ignore")
pd.set_option("mode.chained_assignment", None)


def _axis(frame):
    line = linecache.getline(frame.f_code.co_filename, frame.f_lineno)
    if "get_width" in line:
        return 0
    if "get_height" in line:
        return 1
    raise RuntimeError("keyed random: cannot tell the axis of %r" % line.strip())


class KeyedRandom:
    """Stand-in for the `random` module inside the Environment 2.0 modules."""

    def randint(self, a, b):
        f = sys._getframe(1)
        fn = f.f_code.co_name
        if fn == "<listcomp>" and f.f_back.f_code.co_name in ("create_ostriches", "create_wolves",
                                                              "create_bushes"):
            owner = f.f_back.f_locals["self"]
            if f.f_back.f_locals.get("spawn_positions") != []:
                raise RuntimeError("keyed random: only the all-random create_* path is keyed")
            entity = len(owner._environments) + int(f.f_locals["_"])
            w = owner._world
            site, ep, turn, axis = kr.SITE_T_CREATE, 0, 0, _axis(f)
        elif fn == "_get_random_spawn_indices":
            single = f.f_locals["self"]
            w, entity = single.world, int(single.id)
            site, ep, turn, axis = kr.SITE_T_RESET, w._wab_episode, 0, _axis(f)
        elif fn == "default_game_update":
            w, entity = f.f_locals["self"], int(f.f_locals["entity_id"])
            kind = f.f_locals["entity"]["Type"]
            site = {"Wolf": kr.SITE_T_KILL, "Ostrich": kr.SITE_T_EAT}[kind]
            ep, turn, axis = w._wab_episode, int(w._current_turn), 0
        else:
            raise RuntimeError("keyed random: unexpected randint from %s" % fn)
        ek = kr.episode_key(w._wab_seed, w._wab_world, ep)
        return kr.randint_keyed(ek, site, turn, entity, axis, int(a), int(b))

    def __getattr__(self, name):
        raise RuntimeError("keyed random: random.%s not keyed" % name)


_mods = None


def load_reference():
    """Import the unmodified Environment 2.0 modules with the keyed `random`."""
    global _mods
    if _mods is None:
        sys.path.insert(0, ENV2_DIR)
        import World  # noqa: F401
        import WAB_Environment2
        import WAB_Environment2_Single

        keyed = KeyedRandom()
        for m in (World, WAB_Environment2, WAB_Environment2_Single):
            m.random = keyed
        _mods = {"World": World, "WAB_Environment2": WAB_Environment2,
                 "WAB_Environment2_Single": WAB_Environment2_Single}
    return _mods


def make_env(seed: int, world_id: int, width: int, height: int, game_options=None):
    """A reference `WAB_Environment2(width, height, options)` whose draws are keyed by
    (seed, world_id, episode); reset_environment() counts the episodes."""
    m = load_reference()
    base = m["WAB_Environment2"].WAB_Environment2

    class KeyedEnv2(base):
        def reset_environment(self):
            self._world._wab_episode += 1
            return super().reset_environment()

    opts = dict(m["WAB_Environment2"].default_game_options)
    if game_options:
        opts.update(game_options)
    env = KeyedEnv2(width, height, opts)
    env._world._wab_seed, env._world._wab_world, env._world._wab_episode = seed, world_id, 0
    return env


def record_layout(n_entities: int, n_bushes: int):
    """Byte layout of one observation record (wab_torus.h `wab2_obs`): returns (size, offsets)."""
    N, NB = n_entities, n_bushes
    off = {"food": 0, "x": 8, "y": 12, "visible": 16, "flag": 20, "status": 21, "type": 22,
           "delta": 24, "bush_food": 24 + 2 * N}
    size = (24 + 2 * N + NB + 15) // 16 * 16
    return size, off


TYPE_CODE = {"Ostrich": 0, "Wolf": 1, "Bush": 2}


def encode_obs(obs, entity_id, types, n_bushes, record):
    """The reference's get_obs() result ([visible-objects frame, internal obs list],
    World.py:360-377) into one fixed-size record (uint8 array, zeroed by the caller)."""
    N = len(types)
    size, off = record_layout(N, n_bushes)
    df, internal = obs
    bush0 = N - n_bushes
    vis = 0
    prev = -1
    for _, row in df.iterrows():
        j = int(row["index"])
        if j <= prev:
            raise RuntimeError("visible objects not in entity-id order")
        prev = j
        if row["Type"] != types[j]:
            raise RuntimeError("row type %r != entity %d's %r" % (row["Type"], j, types[j]))
        dx, dy = int(row["Delta_X"]), int(row["Delta_Y"])
        if dx != row["Delta_X"] or dy != row["Delta_Y"] or not (-128 <= dx < 128 and -128 <= dy < 128):
            raise RuntimeError("delta not an int8: %r" % ((row["Delta_X"], row["Delta_Y"]),))
        vis |= 1 << j
        record[off["delta"] + 2 * j] = dx & 0xFF
        record[off["delta"] + 2 * j + 1] = dy & 0xFF
        extra = row["Additional_Data"]
        if types[j] == "Bush":
            (f,) = extra
            if int(f) != f or not 0 <= f <= 255:
                raise RuntimeError("bush food %r not a byte" % (f,))
            record[off["bush_food"] + j - bush0] = int(f)
        elif list(extra) != []:
            raise RuntimeError("unexpected Additional_Data %r" % (extra,))
    t = types[entity_id]
    x, y, food = internal[0], internal[1], internal[2]
    record[off["food"]:off["food"] + 8] = np.frombuffer(np.float64(food).tobytes(), np.uint8)
    record[off["x"]:off["x"] + 4] = np.frombuffer(np.int32(x).tobytes(), np.uint8)
    record[off["y"]:off["y"] + 4] = np.frombuffer(np.int32(y).tobytes(), np.uint8)
    record[off["visible"]:off["visible"] + 4] = np.frombuffer(np.uint32(vis).tobytes(), np.uint8)
    if t == "Ostrich":  # [x, y, food, role, status]   (World.py:50-51)
        record[off["flag"]], record[off["status"]] = int(internal[3]), int(internal[4])
    elif t == "Wolf":   # [x, y, food, is_running, status]  (World.py:80-81)
        record[off["flag"]], record[off["status"]] = int(bool(internal[3])), int(internal[4])
    elif len(internal) != 3:  # bush: [x, y, food]  (World.py:17-18)
        raise RuntimeError("bush internal obs %r" % (internal,))
    record[off["type"]] = TYPE_CODE[t]
    return record
