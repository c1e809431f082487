"""Options of the Environment 2.0 torus world and their C-ABI struct (include/wab_torus.h).

`DEFAULT_GAME_OPTIONS` restates `Environment 2.0/WAB_Environment2.py:9-50` key for key.  World
reads ten of them (World.py:173-226, 365-374); the rest (rewards, modes, wolf speeds and
costs, bush power, viewport size, ...) are never read by the Env 2.0 code and are accepted and
ignored here as they are there.
"""
from __future__ import annotations

import ctypes

DEFAULT_GAME_OPTIONS = {
    # GYM OPTIONS
    "ostrich_mode_or_wolf_mode": 0,
    "reward_per_turn": 0,
    "reward_for_being_killed": -1,
    "reward_for_starving": -1,
    "reward_for_finishing": 1,
    "reward_for_eating": 0,
    "gatherer_only": False,
    "lookout_only": True,
    "restrict_view": False,
    "starting_role": 1,
    # GAME
    "max_turns": 80,
    "num_ostriches": 20,
    "height": 11,
    "width": 11,
    "bush_power": 100,
    "max_berries_per_bush": 200,
    # BUSHES
    "food_per_bush": 20,
    "food_given_per_turn": 5,
    # OSTRICHES
    "ostrich_starting_food": 40.0,
    "ostrich_food_eaten_per_turn": 1.0,
    "ostrich_move_speed": 1.0,
    "lookout_view_radius": 9,
    "gatherer_view_radius": 5,
    # WOLVES
    "num_wolves": 20,
    "wolf_spawn_margin": 1,
    "chance_wolf_on_square": 0.001,
    "wolves": True,
    "wolf_starting_food": 20,
    "wolf_food_for_eating_ostrich": 10,
    "wolves_can_move": True,
    "wolf_walk_speed": 1.0,
    "wolf_walk_cost": 0.1,
    "wolf_run_speed": 2.0,
    "wolf_run_cost": 0.2,
    "wolf_view_radius": 6,
}

MAX_ENTITIES = 32
MAX_OSTRICHES = 8
MAX_SIDE = 127


class Wab2Config(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("num_ostriches", ctypes.c_int32), ("num_wolves", ctypes.c_int32),
                ("num_bushes", ctypes.c_int32), ("starting_role", ctypes.c_int32),
                ("ostrich_starting_food", ctypes.c_double), ("food_per_bush", ctypes.c_int32),
                ("food_given_per_turn", ctypes.c_int32), ("wolf_starting_food", ctypes.c_double),
                ("wolf_food_for_eating_ostrich", ctypes.c_double),
                ("lookout_view_radius", ctypes.c_int32), ("gatherer_view_radius", ctypes.c_int32),
                ("wolf_view_radius", ctypes.c_int32), ("max_turns", ctypes.c_int32),
                ("autoreset", ctypes.c_int32)]


def _int(opts, key, lo, hi):
    v = opts[key]
    if isinstance(v, bool) or float(v) != int(v) or not lo <= int(v) <= hi:
        raise ValueError("%s = %r: an integer in [%d, %d] is required" % (key, v, lo, hi))
    return int(v)


def make_config(width=32, height=32, num_ostriches=1, num_wolves=8, num_bushes=16,
                game_options=None, autoreset=True):
    """(Wab2Config, full options dict) for WAB_Environment2(width, height, game_options) with
    the given entity counts (create_ostriches / create_wolves / create_bushes)."""
    opts = dict(DEFAULT_GAME_OPTIONS)
    if game_options:
        opts.update(game_options)
    for k, v in (("width", width), ("height", height)):
        if isinstance(v, bool) or int(v) != v or not 1 <= int(v) <= MAX_SIDE:
            raise ValueError("world %s = %r: an integer in [1, %d] is required" % (k, v, MAX_SIDE))
    no, nw, nb = int(num_ostriches), int(num_wolves), int(num_bushes)
    if min(no, nw, nb) < 0 or no > MAX_OSTRICHES or no + nw + nb > MAX_ENTITIES or no + nw + nb == 0:
        raise ValueError("entity counts (%d, %d, %d): 0..%d ostriches, at most %d entities in all"
                         % (no, nw, nb, MAX_OSTRICHES, MAX_ENTITIES))
    role = _int(opts, "starting_role", 0, 1)  # World.get_observations knows roles 0 and 1 only
    cfg = Wab2Config(
        width=int(width), height=int(height), num_ostriches=no, num_wolves=nw, num_bushes=nb,
        starting_role=role, ostrich_starting_food=float(opts["ostrich_starting_food"]),
        food_per_bush=_int(opts, "food_per_bush", 0, 255),
        food_given_per_turn=_int(opts, "food_given_per_turn", 0, 255),
        wolf_starting_food=float(opts["wolf_starting_food"]),
        wolf_food_for_eating_ostrich=float(opts["wolf_food_for_eating_ostrich"]),
        lookout_view_radius=_int(opts, "lookout_view_radius", 0, 1 << 20),
        gatherer_view_radius=_int(opts, "gatherer_view_radius", 0, 1 << 20),
        wolf_view_radius=_int(opts, "wolf_view_radius", 0, 1 << 20),
        max_turns=_int(opts, "max_turns", 0, 1 << 30), autoreset=int(bool(autoreset)))
    return cfg, opts


def record_size(n_entities, n_bushes):
    """Bytes of one observation record (include/wab_torus.h)."""
    return (24 + 2 * n_entities + n_bushes + 15) // 16 * 16
