"""ctypes binding of the C oracle (oracle/wab_oracle.c).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The oracle is the checker; the product (wab_gym_amd) never loads it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libwab_oracle.so")

_lib = None


def build(quiet=True):
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def _stale():
    srcs = [os.path.join(HERE, f) for f in ("wab_oracle.c", "wab_oracle.h", "wab_torus_oracle.c", "Makefile")]
    srcs.append(os.path.join(os.path.dirname(HERE), "wab_gym_amd", "csrc", "wab_glyphs.h"))
    srcs.append(os.path.join(os.path.dirname(HERE), "include", "wab.h"))
    srcs.append(os.path.join(os.path.dirname(HERE), "include", "wab_torus.h"))
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.exists(s) and os.path.getmtime(s) > t for s in srcs)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or _stale():
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.wabo_create.restype = P
        L.wabo_create.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64]
        L.wabo_destroy.argtypes = [P]
        L.wabo_num_actions.argtypes = [P]
        L.wabo_reset.argtypes = [P] * 6
        L.wabo_step.argtypes = [P] * 12 + [ctypes.c_int]
        L.wabo_get_state.argtypes = [P] * 7
        L.wabo_episode_key.restype = ctypes.c_uint64
        L.wabo_episode_key.argtypes = [ctypes.c_uint64] * 3
        L.wabo_draw_U.restype = ctypes.c_uint64
        L.wabo_draw_U.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_int64, ctypes.c_uint32]
        L.wabo_spawn_hits.argtypes = [P, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, P, ctypes.c_int]
        L.wabo_gap_threshold.restype = ctypes.c_uint64
        L.wabo_gap_threshold.argtypes = [P, ctypes.c_int]
        L.wabo_feature_dim.argtypes = [ctypes.c_int] * 3
        L.wabo_featurize.argtypes = [ctypes.c_int64] + [ctypes.c_int] * 4 + [P] * 6
        L.wabo_egocentric.argtypes = [P, P]
        L.wabo_superbasic_dim.argtypes = [ctypes.c_int] * 3
        L.wabo_render.argtypes = [ctypes.c_int64] + [ctypes.c_int] * 6 + [P] * 5
        L.wabo_featurize_superbasic.argtypes = [ctypes.c_int64] + [ctypes.c_int] * 4 + [P] * 5
        L.wabo_discounted_returns.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P, ctypes.c_double, P, P, P,
                                              ctypes.c_int]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class OracleBatch:
    """B envs on the host CPU, same array layouts as wab.h's wab_obs."""

    def __init__(self, options=None, batch=1, seed=0x5EED, env_id_base=0, autoreset=True,
                 plane_stride=0):
        from wab_gym_amd.options import make_config  # config translation only (no product code path)

        self.cfg, self._keep = make_config(options, autoreset=autoreset, plane_stride=plane_stride)
        self.options = self._keep[1]
        self.B = int(batch)
        self.W, self.H = self.cfg.width, self.cfg.height
        self.S = plane_stride or self.H
        self.h = lib().wabo_create(ctypes.addressof(self.cfg), self.B, seed, env_id_base)
        if not self.h:
            raise ValueError("oracle rejected the options")
        self.n_actions = lib().wabo_num_actions(self.h)
        shape = (self.B, 3, self.W, self.S)
        self.planes = np.zeros(shape, np.uint8)
        self.food_turns = np.zeros(self.B, np.uint8)
        self.role = np.zeros(self.B, np.uint8)
        self.status = np.zeros(self.B, np.uint8)
        self.reward = np.zeros(self.B, np.float32)
        self.done = np.zeros(self.B, np.uint8)
        self.t_planes = np.zeros(shape, np.uint8)
        self.t_food_turns = np.zeros(self.B, np.uint8)
        self.t_role = np.zeros(self.B, np.uint8)
        self.t_status = np.zeros(self.B, np.uint8)

    def __del__(self):
        if getattr(self, "h", None):
            lib().wabo_destroy(self.h)
            self.h = None

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().wabo_reset(self.h, _p(m), _p(self.planes), _p(self.food_turns), _p(self.role),
                         _p(self.status))
        return self.planes, self.food_turns, self.role, self.status

    def step(self, actions, nthreads=1):
        a = np.ascontiguousarray(actions, dtype=np.int8)
        lib().wabo_step(self.h, _p(a), _p(self.planes), _p(self.food_turns), _p(self.role),
                        _p(self.status), _p(self.reward), _p(self.done), _p(self.t_planes),
                        _p(self.t_food_turns), _p(self.t_role), _p(self.t_status), int(nthreads))
        return self.planes, self.food_turns, self.role, self.status, self.reward, self.done

    def egocentric(self):
        """Bush proximities u8 [B, 5] of the current state (wab_env.py:652-667)."""
        out = np.zeros((self.B, 5), np.uint8)
        lib().wabo_egocentric(self.h, _p(out))
        return out

    def spawn_hits(self, ek, turn, n):
        """The keyed spawn set of n tiles at `turn` (keyed_rng.spawn_hits) under this batch's q."""
        out = np.zeros(max(n, 1), np.int32)
        k = lib().wabo_spawn_hits(self.h, ek, turn, n, _p(out), n)
        return out[:k].tolist()

    def gap_threshold(self, g):
        return int(lib().wabo_gap_threshold(self.h, g))

    def state(self):
        food = np.zeros(self.B, np.float64)
        x = np.zeros(self.B, np.int32)
        y = np.zeros(self.B, np.int32)
        turn = np.zeros(self.B, np.int32)
        nw = np.zeros(self.B, np.int32)
        ep = np.zeros(self.B, np.uint32)
        lib().wabo_get_state(self.h, _p(food), _p(x), _p(y), _p(turn), _p(nw), _p(ep))
        return dict(food=food, x=x, y=y, turn=turn, n_wolves=nw, episode=ep)


def episode_key(seed, env, episode):
    return int(lib().wabo_episode_key(seed, env, episode))


def draw_U(ek, site, turn, x, y, k=0):
    return int(lib().wabo_draw_U(ek, site, turn, x, y, k))


def feature_dim(W, H, turns_empty=40):
    return int(lib().wabo_feature_dim(W, H, turns_empty))


def featurize(planes, food_turns, role, status, view_mask, W, H, turns_empty=40):
    """planes [B,3,W,S] u8, scalars [B] u8, view_mask [B,11,11] u8 -> float32 [B, F]."""
    planes = np.ascontiguousarray(planes, dtype=np.uint8)
    B, S = planes.shape[0], planes.shape[3]
    F = feature_dim(W, H, turns_empty)
    out = np.zeros((B, F), np.float32)
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in (food_turns, role, status, view_mask)]
    lib().wabo_featurize(B, W, H, S, turns_empty, _p(planes), _p(arrs[0]), _p(arrs[1]), _p(arrs[2]),
                         _p(arrs[3]), _p(out))
    return out


def superbasic_dim(W=11, H=11, turns_empty=40):
    return int(lib().wabo_superbasic_dim(W, H, turns_empty))


def featurize_superbasic(planes, food_turns, role, status, W, H, turns_empty=40):
    """SuperBasicObservationWrapper + flatten: planes [B,3,W,S] u8, scalars [B] u8 -> f32 [B, F]."""
    planes = np.ascontiguousarray(planes, dtype=np.uint8)
    B, S = planes.shape[0], planes.shape[3]
    out = np.zeros((B, superbasic_dim(W, H, turns_empty)), np.float32)
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in (food_turns, role, status)]
    lib().wabo_featurize_superbasic(B, W, H, S, turns_empty, _p(planes), _p(arrs[0]), _p(arrs[1]), _p(arrs[2]),
                                    _p(out))
    return out


def render(planes, role, status, W, H, restrict_view=False, scale=32, food_turns=None, draw_health=False):
    """render(mode="rgb_array", scale, draw_health) of observations -> u8 [B, W*s, H*s, 3]
    (draw_health needs food_turns)."""
    planes = np.ascontiguousarray(planes, dtype=np.uint8)
    B, S = planes.shape[0], planes.shape[3]
    out = np.zeros((B, W * scale, H * scale, 3), np.uint8)
    r = np.ascontiguousarray(role, dtype=np.uint8)
    st = np.ascontiguousarray(status, dtype=np.uint8)
    ft = np.ascontiguousarray(np.zeros(B) if food_turns is None else food_turns, dtype=np.uint8)
    if draw_health and food_turns is None:
        raise ValueError("draw_health needs food_turns")
    lib().wabo_render(B, W, H, S, int(bool(restrict_view)), scale, int(bool(draw_health)), _p(planes), _p(ft),
                      _p(r), _p(st), _p(out))
    return out


def discounted_returns(reward, done, gamma=0.99, bootstrap=None, exact_values=None):
    """exact_values: the doubles one step can return (their float32 stands for them)."""
    reward = np.ascontiguousarray(reward, dtype=np.float32)
    done = np.ascontiguousarray(done, dtype=np.uint8)
    T, B = reward.shape
    out = np.zeros((T, B), np.float32)
    bs = None if bootstrap is None else np.ascontiguousarray(bootstrap, dtype=np.float32)
    ev = None if exact_values is None else np.ascontiguousarray(exact_values, dtype=np.float64)
    lib().wabo_discounted_returns(T, B, _p(reward), _p(done), gamma, _p(bs), _p(out), _p(ev),
                                  0 if ev is None else len(ev))
    return out
