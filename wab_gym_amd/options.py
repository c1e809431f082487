"""Game options and their translation into the C-ABI `wab_config` (include/wab.h).

`default_game_options` mirrors the reference's dict field for field
(`wab_env.py:11-39`), including its None-means-random convention for
`starting_food` / `starting_role` (`wab_env.py:596-599`) and the hidden `god_mode`
key read with `.get` (`wab_env.py:292`).
"""
from __future__ import annotations

import ctypes

import numpy as np

default_game_options = {
    # GYM OPTIONS
    "reward_per_turn": 0,
    "reward_for_being_killed": -1,
    "reward_for_starving": -1,
    "reward_for_finishing": 1,
    "reward_for_eating": 0.1,
    "gatherer_only": False,
    "lookout_only": True,
    "restrict_view": False,
    "starting_role": 1,
    # GAME
    "max_turns": 80,
    "num_ostriches": 1,  # ignored by the reference too: spawn_ostriches adds one (wab_env.py:595-611)
    "height": 11,
    "width": 11,
    "bush_power": 100,
    "max_berries_per_bush": 200,
    # FOOD
    "turns_to_fill_food": 8,
    "turns_to_empty_food": 40,
    "starting_food": 1,
    # WOLVES
    "wolf_spawn_margin": 1,
    "chance_wolf_on_square": 0.001,
    "wolf_chance_to_despawn": 0.05,
    "wolves": True,
    "wolves_can_move": True,
}

WOLF_SLOTS = (8, 16, 32)
MAX_VIEW = 63


class WabConfig(ctypes.Structure):
    """ctypes mirror of `wab_config` (include/wab.h); field order is the ABI."""

    _fields_ = [
        ("reward_per_turn", ctypes.c_double),
        ("reward_for_being_killed", ctypes.c_double),
        ("reward_for_starving", ctypes.c_double),
        ("reward_for_finishing", ctypes.c_double),
        ("reward_for_eating", ctypes.c_double),
        ("gatherer_only", ctypes.c_int32),
        ("lookout_only", ctypes.c_int32),
        ("restrict_view", ctypes.c_int32),
        ("starting_role", ctypes.c_int32),
        ("starting_role_random", ctypes.c_int32),
        ("starting_food_random", ctypes.c_int32),
        ("starting_food", ctypes.c_double),
        ("max_turns", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("max_berries_per_bush", ctypes.c_int32),
        ("bush_power", ctypes.c_double),
        ("turns_to_fill_food", ctypes.c_int32),
        ("turns_to_empty_food", ctypes.c_int32),
        ("wolf_spawn_margin", ctypes.c_int32),
        ("chance_wolf_on_square", ctypes.c_double),
        ("wolf_chance_to_despawn", ctypes.c_double),
        ("wolves", ctypes.c_int32),
        ("wolves_can_move", ctypes.c_int32),
        ("god_mode", ctypes.c_int32),
        ("autoreset", ctypes.c_int32),
        ("plane_stride", ctypes.c_int32),
        ("eaten_capacity", ctypes.c_int32),
        ("wolf_slots", ctypes.c_int32),
        ("bush_thresholds", ctypes.POINTER(ctypes.c_uint64)),
    ]


def bush_thresholds(bush_power, max_berries_per_bush) -> np.ndarray:
    """T_k, k = 1..max_berries: the smallest 53-bit U whose u = U*2^-53 gives a bush value
    >= k under the reference's own numpy expression
    `np.round(u ** bush_power * max_berries_per_bush)` (`wab_env.py:632-635`).

    Bisection over the 2^53 grid of doubles a 53-bit random draw can take, evaluated
    with the same numpy array arithmetic the reference uses, so a kernel that compares
    U against this table reproduces the reference's rounding bit for bit
    (the value is monotone in u; tests/test_thresholds.py checks every boundary).
    A value no draw reaches gets 2^53.
    """
    n = int(max_berries_per_bush)
    if n <= 0:
        return np.zeros(0, dtype=np.uint64)
    k = np.arange(1, n + 1, dtype=np.float64)
    lo = np.zeros(n, dtype=np.int64)            # f(lo) < k
    hi = np.full(n, 1 << 53, dtype=np.int64)    # f(hi) >= k (2^53 = "never")

    def f(U):
        u = U.astype(np.float64) * (2.0 ** -53)
        return np.round(u ** bush_power * max_berries_per_bush)

    while True:
        open_ = hi - lo > 1
        if not open_.any():
            break
        mid = (lo + hi) // 2
        ge = f(mid) >= k
        hi = np.where(open_ & ge, mid, hi)
        lo = np.where(open_ & ~ge, mid, lo)
    return hi.astype(np.uint64)


def _opt(options, key):
    if key == "god_mode":
        return options.get("god_mode")
    return options[key]


def validate(options):
    W, H = int(options["width"]), int(options["height"])
    if W % 2 == 0 or H % 2 == 0:
        raise ValueError("width and height must be odd numbers")  # wab_env.py:147-148
    if W > MAX_VIEW or H > MAX_VIEW or W < 1 or H < 1:
        raise ValueError("width/height must be in [1, %d]" % MAX_VIEW)
    if options["restrict_view"] and (W < 11 or H < 11):
        raise ValueError("restrict_view indexes 11x11 masks into the grid (wab_env.py:354-355)")
    if not 0 <= int(options["max_berries_per_bush"]) <= 255:
        raise ValueError("max_berries_per_bush must be in [0, 255]")


def make_config(options=None, autoreset=True, plane_stride=0, eaten_capacity=0, wolf_slots=0):
    """Build a `WabConfig`; returns (config, keepalive) — keep `keepalive` referenced."""
    opts = dict(default_game_options)
    if options:
        opts.update(options)
    validate(opts)
    table = np.ascontiguousarray(bush_thresholds(opts["bush_power"], opts["max_berries_per_bush"]))
    c = WabConfig()
    for key in ("reward_per_turn", "reward_for_being_killed", "reward_for_starving",
                "reward_for_finishing", "reward_for_eating"):
        setattr(c, key, float(opts[key]))
    c.gatherer_only = int(bool(opts["gatherer_only"]))
    c.lookout_only = int(bool(opts["lookout_only"]))
    c.restrict_view = int(bool(opts["restrict_view"]))
    c.starting_role_random = int(opts["starting_role"] is None)
    c.starting_role = 0 if opts["starting_role"] is None else int(opts["starting_role"])
    c.starting_food_random = int(opts["starting_food"] is None)
    c.starting_food = 0.0 if opts["starting_food"] is None else float(opts["starting_food"])
    c.max_turns = int(opts["max_turns"])
    c.height = int(opts["height"])
    c.width = int(opts["width"])
    c.max_berries_per_bush = int(opts["max_berries_per_bush"])
    c.bush_power = float(opts["bush_power"])
    c.turns_to_fill_food = int(opts["turns_to_fill_food"])
    c.turns_to_empty_food = int(opts["turns_to_empty_food"])
    c.wolf_spawn_margin = int(opts["wolf_spawn_margin"])
    c.chance_wolf_on_square = float(opts["chance_wolf_on_square"])
    c.wolf_chance_to_despawn = float(opts["wolf_chance_to_despawn"])
    c.wolves = int(bool(opts["wolves"]))
    c.wolves_can_move = int(bool(opts["wolves_can_move"]))
    c.god_mode = int(bool(_opt(opts, "god_mode")))
    c.autoreset = int(bool(autoreset))
    c.plane_stride = int(plane_stride)
    c.eaten_capacity = int(eaten_capacity)
    c.wolf_slots = int(wolf_slots)
    c.bush_thresholds = table.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    return c, (table, opts)


def n_actions(options) -> int:
    """Action-table size (wab_env.py:149-182)."""
    if options["gatherer_only"] or options["lookout_only"]:
        return 5
    return 6


LOOKOUT_MASK = np.array(
    [[1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1], [1, 1, 0, 0, 0, 0, 0, 0, 0, 1, 1],
     [1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1], [0] * 11, [0] * 11, [0] * 11, [0] * 11, [0] * 11,
     [1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1], [1, 1, 0, 0, 0, 0, 0, 0, 0, 1, 1],
     [1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1]], dtype=np.uint8)  # wab_env.py:109-123
GATHERER_MASK = np.array(
    [[1] * 11, [1] * 11, [1] * 11, [1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1],
     [1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1], [1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1],
     [1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 1], [1, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1],
     [1] * 11, [1] * 11, [1] * 11], dtype=np.uint8)  # wab_env.py:125-139


def view_masks(options) -> np.ndarray:
    """[2, 11, 11] view_mask indexed by role (wab_env.py:360-368): zeros unless restrict_view."""
    if not options["restrict_view"]:
        return np.zeros((2, 11, 11), dtype=np.uint8)
    return np.stack([LOOKOUT_MASK, GATHERER_MASK])
