"""Replay a golden fixture (tests/golden/*.npz) through a backend and compare bit for bit.

A backend is a factory `make(options, env_id_base, batch, autoreset, plane_stride)` returning
an object with
    reset()          -> (planes [B,3,W,S] u8, food_turns, role, status)        numpy
    step(actions)    -> (planes, food_turns, role, status, reward f32, done u8,
                         terminal (planes, food_turns, role, status) or None)   numpy
    state()          -> dict(food, x, y, n_wolves, ...) or None
The golden protocol is described in tests/golden/make_golden.py.
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ["default", "continue", "wide31", "neither6", "gatherer", "static_god", "nowolves",
        "rand_start", "wolfy", "restrict", "rect9x13"]


def load(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(bytes(d["meta"]).decode())
    return d


def unpack(bits, W, H):
    """packed bits [..., nbytes] -> planes [..., 3, W, H]"""
    n = 3 * W * H
    flat = np.unpackbits(bits, axis=-1)[..., :n]
    return flat.reshape(bits.shape[:-1] + (3, W, H))


def groups(env_ids):
    """split env ids into runs of consecutive ids: [(first_index, base, length)]"""
    out, i = [], 0
    while i < len(env_ids):
        j = i
        while j + 1 < len(env_ids) and env_ids[j + 1] == env_ids[j] + 1:
            j += 1
        out.append((i, env_ids[i], j - i + 1))
        i = j + 1
    return out


class Mismatch(AssertionError):
    pass


def _cmp(what, got, want, t, e0):
    if not np.array_equal(got, want):
        bad = np.argwhere(np.asarray(got != want).reshape(len(got), -1).any(axis=1))[:, 0]
        raise Mismatch("%s differs at t=%s for envs %s (first: got %r want %r)" % (
            what, t, (bad + e0).tolist()[:8], np.asarray(got)[bad[0]].ravel()[:16],
            np.asarray(want)[bad[0]].ravel()[:16]))


def replay(name, make, plane_stride=0, check_state=True, max_steps=None):
    g = load(name)
    meta = g["meta"]
    W, H = meta["width"], meta["height"]
    S = plane_stride or H
    T = meta["T"] if max_steps is None else min(meta["T"], max_steps)
    autoreset = meta["protocol"] == "autoreset"
    opts = meta["options"]
    steps = 0
    for e0, base, n in groups(meta["env_ids"]):
        sl = slice(e0, e0 + n)
        be = make(opts, base, n, autoreset, plane_stride)
        planes, food, role, status = be.reset()
        _check_obs("reset", (planes, food, role, status), g["reset0_bits"][sl],
                   g["reset0_scalars"][sl], W, H, S, -1, e0)
        for t in range(T):
            a = g["actions"][t, sl]
            planes, food, role, status, reward, done, term = be.step(a)
            gdone = g["done"][t, sl]
            _cmp("done", done.astype(bool), gdone, t, e0)
            _cmp("reward", reward.astype(np.float32), g["reward"][t, sl].astype(np.float32), t, e0)
            if autoreset:
                d = gdone
                if term is not None and d.any():
                    _check_obs("terminal", tuple(x[d] for x in term), g["bits"][t, sl][d],
                               g["scalars"][t, sl][d], W, H, S, t, e0)
                bits = np.where(d[:, None], g["rbits"][t, sl], g["bits"][t, sl])
                sc = np.where(d[:, None], g["rscalars"][t, sl], g["scalars"][t, sl])
            else:
                d = np.zeros(n, bool)
                bits, sc = g["bits"][t, sl], g["scalars"][t, sl]
            _check_obs("obs", (planes, food, role, status), bits, sc, W, H, S, t, e0)
            if check_state:
                st = be.state()
                if st is not None:
                    nd = ~d
                    _cmp("food(f64)", st["food"][nd].view(np.uint64),
                         g["food"][t, sl][nd].view(np.uint64), t, e0)
                    _cmp("pos", np.stack([st["x"], st["y"]], 1)[nd], g["pos"][t, sl][nd], t, e0)
                    _cmp("n_wolves", st["n_wolves"][nd], g["n_wolves"][t, sl][nd], t, e0)
            steps += n
    return steps


def replay_rollout(name, make, plane_stride=0, segments=(1, 7, 64)):
    """Replay a golden set through a multi-step backend: `make(...)` as for replay(), with
    reset() as there and rollout(actions [n, B]) -> per step (planes, food_turns, role, status,
    reward, done) numpy arrays [n, ...].  The set's T steps run as consecutive rollouts of the
    lengths in `segments` (cycled; state carried across calls), every step compared with the
    golden obs/reward/done, and the hidden state after every rollout with the golden state of
    its last step (envs that did not just finish)."""
    g = load(name)
    meta = g["meta"]
    W, H = meta["width"], meta["height"]
    S = plane_stride or H
    T = meta["T"]
    autoreset = meta["protocol"] == "autoreset"
    steps = 0
    for e0, base, n in groups(meta["env_ids"]):
        sl = slice(e0, e0 + n)
        be = make(meta["options"], base, n, autoreset, plane_stride)
        planes, food, role, status = be.reset()
        _check_obs("reset", (planes, food, role, status), g["reset0_bits"][sl],
                   g["reset0_scalars"][sl], W, H, S, -1, e0)
        t0, k = 0, 0
        while t0 < T:
            L = min(segments[k % len(segments)], T - t0)
            k += 1
            planes, food, role, status, reward, done = be.rollout(g["actions"][t0:t0 + L, sl])
            for i in range(L):
                t = t0 + i
                gdone = g["done"][t, sl]
                _cmp("done", done[i].astype(bool), gdone, t, e0)
                _cmp("reward", reward[i].astype(np.float32), g["reward"][t, sl].astype(np.float32), t, e0)
                d = gdone if autoreset else np.zeros(n, bool)
                bits = np.where(d[:, None], g["rbits"][t, sl], g["bits"][t, sl])
                sc = np.where(d[:, None], g["rscalars"][t, sl], g["scalars"][t, sl])
                _check_obs("rollout obs", (planes[i], food[i], role[i], status[i]), bits, sc, W, H, S, t, e0)
            t = t0 + L - 1
            st = be.state()
            nd = ~(g["done"][t, sl].astype(bool) if autoreset else np.zeros(n, bool))
            _cmp("food(f64)", st["food"][nd].view(np.uint64), g["food"][t, sl][nd].view(np.uint64), t, e0)
            _cmp("pos", np.stack([st["x"], st["y"]], 1)[nd], g["pos"][t, sl][nd], t, e0)
            _cmp("n_wolves", st["n_wolves"][nd], g["n_wolves"][t, sl][nd], t, e0)
            t0 += L
            steps += n * L
    return steps


def _check_obs(what, obs, bits, scalars, W, H, S, t, e0):
    planes, food, role, status = obs
    want = unpack(bits, W, H)
    got = np.asarray(planes)
    if S != H:
        if got[..., H:].any():
            raise Mismatch("%s: padding bytes not zero at t=%s" % (what, t))
        got = got[..., :H]
    _cmp(what + ".planes", got, want, t, e0)
    _cmp(what + ".food_turns", np.asarray(food), scalars[:, 0], t, e0)
    _cmp(what + ".role", np.asarray(role), scalars[:, 1], t, e0)
    _cmp(what + ".status", np.asarray(status), scalars[:, 2], t, e0)
