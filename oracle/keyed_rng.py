"""Keyed, counter-based random draws — numpy twin of the RNG the HIP kernel uses.

TEST INFRASTRUCTURE (oracle/): imported only by tests/, the golden-vector harness,
`__graft_entry__.smoke()` and bench.py's cpu_baseline leg.  Never on the product path.

Why it exists
-------------
The reference draws every random number from numpy's global MT19937 and consumes
the stream in CPython `set` iteration order (`wab_env.py:566-567`, `:624-625`), so
its trajectories cannot be reproduced by any batched implementation.  Parity is
therefore defined under a *keyed* RNG: each draw the reference makes is replaced
by a pure function of what the draw is *about* (SURVEY.md §8c):

    u(seed, env, episode, site, turn, x, y, k)  ->  53-bit double in [0, 1)

Call sites in the reference and the key they get (site ids):
  1  bush value        `generate_n_bush_values` (`wab_env.py:631-635`)   turn=0, tile (x, y), k=0
  2  wolf spawn        `initialize_wolves` / `spawn_wolves` (`:578-593`, `:527-576`)
                                                                       turn=current_turn, tile, k=0
  3  wolf despawn      `step` (`:262-264`)   turn, wolf tile, k = occurrence index of that tile
                                             among the wolves in list order
  4  starting food     `spawn_ostriches` (`:597`, only if starting_food is None)  tile (0, 0)
  5  starting role     `spawn_ostriches` (`:599`, randint(2))                    tile (0, 0)

Definition (all arithmetic mod 2^64 / 2^32):
    mix64(z)    = splitmix64 finaliser
    ek          = mix64(mix64(mix64(seed + GOLDEN64) ^ env) ^ episode)
    b0, b1      = low / high 32 bits of ek
    xy          = (x & 0xFFFF) | (y & 0xFFFF) << 16
    ts          = site & 0xF | (k & 0xFF) << 4 | (turn & 0xFFFFF) << 12
    h1          = fmix32(xy ^ b0)                     (murmur3 finaliser)
    hi          = fmix32(h1 ^ ts ^ b1)
    lo          = fmix32(h1 ^ rotl32(ts, 16) ^ b0 ^ 0x9E3779B9)
    U           = hi << 21 | lo >> 11                 (53-bit integer)
    u           = U * 2^-53
Every comparison the reference makes against u (`u > 0.05`, `u < 0.0005`, the bush
power-law) is turned into an exact integer comparison on U — see `thresholds`.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
GOLDEN64 = 0x9E3779B97F4A7C15

SITE_BUSH = 1
SITE_SPAWN = 2
SITE_DESPAWN = 3
SITE_START_FOOD = 4
SITE_START_ROLE = 5


def mix64(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def episode_key(seed: int, env: int, episode: int) -> int:
    a = mix64((seed + GOLDEN64) & M64)
    b = mix64(a ^ (env & M64))
    return mix64(b ^ (episode & M64))


def fmix32(h):
    h = np.asarray(h, dtype=np.uint32)
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        h = h ^ (h >> np.uint32(16))
    return h


def _rotl32(v, r):
    v = np.asarray(v, dtype=np.uint32)
    return (v << np.uint32(r)) | (v >> np.uint32(32 - r))


def draw_U(ek: int, site: int, turn, x, y, k=0) -> np.ndarray:
    """53-bit integers U (uint64) for arrays of (turn, x, y, k) under one episode key."""
    x = np.asarray(x, dtype=np.int64)
    y = np.asarray(y, dtype=np.int64)
    turn = np.broadcast_to(np.asarray(turn, dtype=np.int64), x.shape)
    k = np.broadcast_to(np.asarray(k, dtype=np.int64), x.shape)
    b0 = np.uint32(ek & 0xFFFFFFFF)
    b1 = np.uint32(ek >> 32)
    xy = ((x & 0xFFFF) | ((y & 0xFFFF) << 16)).astype(np.uint32)
    ts = ((site & 0xF) | ((k & 0xFF) << 4) | ((turn & 0xFFFFF) << 12)).astype(np.uint32)
    h1 = fmix32(xy ^ b0)
    hi = fmix32(h1 ^ ts ^ b1)
    lo = fmix32(h1 ^ _rotl32(ts, 16) ^ b0 ^ np.uint32(0x9E3779B9))
    return (hi.astype(np.uint64) << np.uint64(21)) | (lo.astype(np.uint64) >> np.uint64(11))


def draw_u(ek: int, site: int, turn, x, y, k=0) -> np.ndarray:
    return draw_U(ek, site, turn, x, y, k).astype(np.float64) * (2.0 ** -53)


# ----------------------------------------------------------------------------------------
# exact integer thresholds for the comparisons the reference makes on u
# ----------------------------------------------------------------------------------------
TWO53 = 1 << 53


def keep_threshold_gt(p: float) -> int:
    """u > p  <=>  U > floor(p * 2^53)   (p*2^53 is exact: power-of-two scaling)."""
    return int(np.floor(np.float64(p) * TWO53))


def hit_threshold_lt(p: float) -> int:
    """u < p  <=>  U < ceil(p * 2^53)."""
    return int(np.ceil(np.float64(p) * TWO53))


def bush_value_from_u(u, power, max_berries):
    """The reference's arithmetic, `wab_env.py:632-635`, evaluated by numpy on arrays."""
    return np.round(np.asarray(u, dtype=np.float64) ** power * max_berries)
