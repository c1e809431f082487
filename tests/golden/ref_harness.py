"""Run the *real* reference `wab_env.py` under a keyed RNG (container-only).

TEST INFRASTRUCTURE.  Used by `make_golden.py` to produce the committed fixtures in
`tests/golden/*.npz`, and by the CPU test-suite only when `/root/reference` exists.
Nothing here runs on the GPU box.

Three shims make the unmodified 2020 reference importable offline:
  1. `shims/gym`: gym 0.17.2 stand-in (not installed, no network).
  2. pandas-1.1 compatibility on pandas 2.x: `DataFrame.append` (`wab_env.py:570,587,601,629`),
     positional `drop(label, 1)` (`:58`), and 1.1's silent fallback when `dtype=int` meets
     `None` in the action tables (`:150-182`), which leaves `role` as float NaN (`:257`).
  3. keyed RNG: `wab_env.np` is replaced by a namespace that forwards everything to numpy
     except `random`, whose draws are computed by `oracle/keyed_rng.py` from the caller's
     frame (what the draw is about), not from a global stream.  Each env instance carries
     (seed, env_id, episode); episode = number of `reset()` calls so far (0 for the one
     the constructor makes, `wab_env.py:186`).
"""
from __future__ import annotations

import os
import sys
import types
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = os.environ.get("WAB_REFERENCE", "/root/reference")

sys.path.insert(0, os.path.join(HERE, "shims"))
sys.path.insert(0, REPO)

import pandas as pd  # noqa: E402

from oracle import keyed_rng as kr  # noqa: E402

warnings.filterwarnings("ignore")
pd.set_option("mode.chained_assignment", None)


# --------------------------------------------------------------------------- pandas 1.1 compat
def _append(self, other, ignore_index=False, **_):
    if isinstance(other, dict):
        other = pd.DataFrame([other])
    if len(self.columns) and len(self) == 0:
        # pandas 1.1: appending to an empty frame keeps its column order
        cols = list(self.columns) + [c for c in other.columns if c not in self.columns]
        out = pd.concat([self.astype(object), other], ignore_index=ignore_index)
        return out[cols].infer_objects()
    return pd.concat([self, other], ignore_index=ignore_index)


_orig_drop = pd.DataFrame.drop


def _drop(self, labels=None, *args, **kwargs):
    if args:
        kwargs.setdefault("axis", args[0])
    return _orig_drop(self, labels, **kwargs)


pd.DataFrame.append = _append
pd.DataFrame.drop = _drop


def _frame(*args, **kwargs):
    try:
        return pd.DataFrame(*args, **kwargs)
    except (ValueError, TypeError, pd.errors.IntCastingNaNError):
        kwargs.pop("dtype", None)
        return pd.DataFrame(*args, **kwargs)


pd_proxy = types.SimpleNamespace(**{k: getattr(pd, k) for k in dir(pd) if not k.startswith("__")})
pd_proxy.DataFrame = _frame


# --------------------------------------------------------------------------- keyed numpy.random
class _KeyedRandom:
    def _owner(self, frame):
        f = frame
        while f is not None:
            s = f.f_locals.get("self")
            if s is not None and hasattr(s, "_wab_key"):
                return s
            f = f.f_back
        raise RuntimeError("keyed RNG: no keyed env on the call stack")

    def random(self, size=None):
        frame = sys._getframe(1)
        fn = frame.f_code.co_name
        env = self._owner(frame)
        ek = env._wab_key()
        if fn == "generate_n_bush_values":
            nb = frame.f_back.f_locals["new_bushes"]
            xs, ys = _ints(nb["x"]), _ints(nb["y"])
            u = kr.draw_u(ek, kr.SITE_BUSH, 0, xs, ys, 0)
        elif fn in ("initialize_wolves", "spawn_wolves"):
            u = _spawn_draws(env, ek, fn, frame.f_locals["new_wolves"])
        elif fn == "step":
            w = env.wolves
            xs, ys = _ints(w["x"]), _ints(w["y"])
            seen = {}
            ks = np.empty(len(xs), dtype=np.int64)
            for i, t in enumerate(zip(xs.tolist(), ys.tolist())):
                ks[i] = seen.get(t, 0)
                seen[t] = ks[i] + 1
            u = kr.draw_u(ek, kr.SITE_DESPAWN, int(env.current_turn), xs, ys, ks)
        elif fn == "spawn_ostriches" and size is None:
            return float(kr.draw_u(ek, kr.SITE_START_FOOD, 0, [0], [0], 0)[0])
        else:
            raise RuntimeError("keyed RNG: unexpected np.random.random call from %s" % fn)
        n = 1 if size is None else int(np.prod(size))
        if len(u) != n:
            raise RuntimeError("keyed RNG: %s asked %d draws, keyed %d" % (fn, n, len(u)))
        return u

    def randint(self, n, *a, **k):
        frame = sys._getframe(1)
        env = self._owner(frame)
        if frame.f_code.co_name != "spawn_ostriches" or a or k:
            raise RuntimeError("keyed RNG: unexpected randint")
        u = kr.draw_u(env._wab_key(), kr.SITE_START_ROLE, 0, [0], [0], 0)[0]
        return int(np.floor(u * n))

    def __getattr__(self, name):
        raise RuntimeError("keyed RNG: np.random.%s not keyed" % name)


def _ints(series):
    return np.rint(np.asarray(series, dtype=np.float64)).astype(np.int64)


def _spawn_draws(env, ek, fn, new_wolves):
    """The per-tile uniforms of initialize_wolves / spawn_wolves (`wab_env.py:578-593`,
    `:527-576`), drawn conditionally on the keyed spawn set (keyed_rng.spawn_hits): the set
    over the view cells at turn 0, or over the ring around the ostrich at the current turn."""
    o = env.game_options
    W, H = int(o["width"]), int(o["height"])
    turn = int(env.current_turn)
    T = kr.hit_threshold_lt(o["chance_wolf_on_square"] / 2)
    ox, oy = (int(round(float(v))) for v in (env.ostriches.iloc[0].x, env.ostriches.iloc[0].y))
    xs, ys = _ints(new_wolves["x"]), _ints(new_wolves["y"])
    if fn == "initialize_wolves":
        idx = [kr.view_index(x - ox, y - oy, W, H) for x, y in zip(xs.tolist(), ys.tolist())]
        n = W * H
    else:
        m = int(o["wolf_spawn_margin"])
        idx = [kr.ring_index(x - ox, y - oy, W, H, m) for x, y in zip(xs.tolist(), ys.tolist())]
        n = (W + 2 * m) * (H + 2 * m) - W * H
    if sorted(idx) != list(range(n)):
        raise RuntimeError("keyed RNG: %s tiles are not the %d-tile canonical set" % (fn, n))
    hits = set(kr.spawn_hits(ek, turn, n, kr.gap_thresholds(T, kr.GAP_CHUNK)))
    V = kr.draw_U(ek, kr.SITE_SPAWN, turn, xs, ys, 0)
    U = [kr.conditional_spawn_U(int(v), T, i in hits) for v, i in zip(V.tolist(), idx)]
    return np.asarray(U, dtype=np.float64) * 2.0 ** -53


np_proxy = types.SimpleNamespace(**{k: getattr(np, k) for k in dir(np) if not k.startswith("__")})
np_proxy.random = _KeyedRandom()

# --------------------------------------------------------------------------- import the reference
_wab_env = None


def load_reference():
    global _wab_env
    if _wab_env is None:
        sys.path.insert(0, REFERENCE)
        import wab_env  # the unmodified reference module

        wab_env.np = np_proxy
        wab_env.pd = pd_proxy
        _wab_env = wab_env
    return _wab_env


def make_env(seed: int, env_id: int, game_options=None, cls="WolvesAndBushesEnv"):
    """A reference `WolvesAndBushesEnv` (or the subclass named `cls`, e.g.
    "WolvesAndBushesEnvEgoCentric") whose draws are keyed by (seed, env_id, episode)."""
    wab_env = load_reference()

    class KeyedEnv(getattr(wab_env, cls)):
        def __init__(self, game_options):
            self._seed, self._env_id, self._episode = seed, env_id, -1
            super().__init__(game_options=game_options)

        def _wab_key(self):
            return kr.episode_key(self._seed, self._env_id, self._episode)

        def reset(self):
            self._episode += 1
            return super().reset()

    opts = dict(wab_env.default_game_options)
    if game_options:
        opts.update(game_options)
    return KeyedEnv(opts)


def obs_arrays(obs):
    """Reference 7-tuple -> (planes u8 [3, W, H], food_turns, role, status)."""
    planes = np.stack([np.asarray(obs[0]), np.asarray(obs[1]), np.asarray(obs[2])]).astype(np.uint8)
    return planes, int(obs[3]), int(obs[4]), int(obs[5])
