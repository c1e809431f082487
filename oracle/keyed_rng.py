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
  6  spawn gaps        the wolf-spawn draws of sites 2 (below), turn, "tile" (k, 0) = k-th gap

Wolf spawns (site 2) are drawn as a *set*, not tile by tile.  The reference draws one
uniform per candidate tile and spawns a wolf where u < q (`:573`, `:590`): iid
Bernoulli(q) over the tiles.  The same joint law is drawn here by geometric gaps over a
canonical tile order (the ring order `ring_index`, or the view-cell order `view_index`
for `initialize_wolves`): the number of misses before the next hit among the m tiles left
is G = #{g in 1..m : U_k < P[g]}, P[g] = floor((1 - q)^g * 2^53) (`gap_thresholds`), with
U_k the site-6 draw of the k-th gap; G = m ends the set (`spawn_hits`; the tiles are
taken in chunks of 128, each its own sequence, so that P is a 129-entry table).  A step with no
spawn (~97.6 % at the defaults) costs ONE draw instead of one per ring tile.  The
per-tile uniforms the reference sees are then drawn conditionally on the set
(`conditional_spawn_U`: below q on a hit tile, at or above q elsewhere, each from the
tile's own site-2 draw), so the reference's comparison returns exactly the set and the
vector it receives is still iid U(0, 1) (to the 2^-53 grid).

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
SITE_GAP = 6
# Environment 2.0 torus world (`Environment 2.0/WAB_Environment2.py`, `World.py`): its draws are
# Python `random.randint(a, b)` calls, keyed per world (env = world id, episode = number of
# reset_environment() calls so far, 0 for the create_* positions)
SITE_T_CREATE = 7   # create_* spawn position      (WAB_Environment2.py:64-106)  tile (entity id, axis)
SITE_T_RESET = 8    # reset spawn position         (WAB_Environment2_Single.py:43-48)  tile (entity id, axis)
SITE_T_EAT = 9      # eat tie-break among bushes   (World.py:125)  turn, tile (ostrich id, 0)
SITE_T_KILL = 10    # kill tie-break among ostriches (World.py:112)  turn, tile (wolf id, 0)


def randint_keyed(ek: int, site: int, turn: int, x: int, y: int, a: int, b: int) -> int:
    """Python's `random.randint(a, b)` (both ends included) under the keyed RNG:
    a + floor(U * (b - a + 1) / 2^53), in exact integer arithmetic."""
    U = int(draw_U(ek, site, turn, [x], [y], 0)[0])
    return a + ((U * (b - a + 1)) >> 53)


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


# ----------------------------------------------------------------------------------------
# wolf spawns as a set: geometric gaps (site 6) over a canonical tile order
# ----------------------------------------------------------------------------------------
def gap_thresholds(T: int, n: int) -> list:
    """P[g], g = 0..n: floor((1 - q)^g * 2^53), q = T * 2^-53 (T = hit_threshold_lt(p)).

    The power is a running product in IEEE double (1 - q is exact), the scaling by 2^53
    exact, so C (wab_capi.hip, wab_oracle.c) and Python get the same integers."""
    omq = float(TWO53 - T) * 2.0 ** -53
    out = [TWO53]
    p = 1.0
    for _ in range(n):
        p = p * omq
        out.append(int(np.floor(p * float(TWO53))))
    return out


def gap_count(U: int, P: list, m: int) -> int:
    """Misses before the next hit among m tiles: #{g in 1..m : U < P[g]} (m: no hit)."""
    lo, hi = 0, m  # P[0] = 2^53 > U; P is non-increasing
    while lo < hi:
        mid = (lo + hi + 1) >> 1
        if U < P[mid]:
            lo = mid
        else:
            hi = mid - 1
    return lo


GAP_CHUNK = 128  # tiles per gap sequence: P is needed for g <= 128 only (a small table)


def spawn_hits(ek: int, turn: int, n: int, P: list) -> list:
    """Ascending indices in [0, n) of the tiles that spawn a wolf at `turn` (iid Bernoulli(q)).

    The tiles are taken in chunks of GAP_CHUNK, each its own gap sequence: the k-th draw of
    chunk c is the site-6 draw of "tile" (k, c).  P = gap_thresholds(T, >= GAP_CHUNK)."""
    hits = []
    for c in range((n + GAP_CHUNK - 1) // GAP_CHUNK):
        base = c * GAP_CHUNK
        m = min(GAP_CHUNK, n - base)
        pos, k = 0, 0
        while pos < m:
            U = int(draw_U(ek, SITE_GAP, turn, [k], [c], 0)[0])
            G = gap_count(U, P, m - pos)
            if G >= m - pos:
                break
            pos += G
            hits.append(base + pos)
            pos += 1
            k += 1
    return hits


def ring_index(dx: int, dy: int, W: int, H: int, margin: int) -> int:
    """Index of the spawn-ring tile at offset (dx, dy) from the ostrich: the bands of rows
    below and above the view first (`margin` rows each, x fastest), then the columns left
    and right of it (y fastest); the order of the kernels' ring table (wab_capi.hip)."""
    m, Wm = margin, W + 2 * margin
    xi, yi = dx + W // 2 + m, dy + H // 2 + m
    if yi < m:
        return yi * Wm + xi
    if yi >= m + H:
        return (yi - H) * Wm + xi
    band = xi if xi < m else xi - W
    return 2 * m * Wm + band * H + (yi - m)


def view_index(dx: int, dy: int, W: int, H: int) -> int:
    """Obs cell i * H + j of the tile at offset (dx, dy) = (W//2 - i, H//2 - j)."""
    return (W // 2 - dx) * H + (H // 2 - dy)


def conditional_spawn_U(V: int, T: int, hit: bool) -> int:
    """A tile's 53-bit uniform given the set: from its own site-2 draw V, below T on a hit
    tile, at or above T elsewhere (uniform on either side to the 2^-53 grid)."""
    return (V * T) >> 53 if hit else T + ((V * (TWO53 - T)) >> 53)
