"""ctypes binding of the torus-world C oracle (oracle/wab_torus_oracle.c).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product (wab_gym_amd) never loads it.
"""
from __future__ import annotations

import ctypes

import numpy as np

from oracle.oracle import _p, lib


def _lib():
    L = lib()
    if not getattr(L, "_torus_typed", False):
        P = ctypes.c_void_p
        L.wabt_create.restype = P
        L.wabt_create.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64]
        L.wabt_destroy.argtypes = [P]
        L.wabt_reset.argtypes = [P, P]
        L.wabt_create_at.restype = P
        L.wabt_create_at.argtypes = [P, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64, P]
        L.wabt_reset_at.argtypes = [P, P, P]
        L.wabt_step.argtypes = [P] * 6 + [ctypes.c_int]
        L.wabt_get_state.argtypes = [P] * 8
        L.wabt_record_size.argtypes = [P]
        L._torus_typed = True
    return L


class OracleTorus:
    """B torus worlds on the host CPU, same array layouts as wab_torus.h."""

    def __init__(self, width=32, height=32, num_ostriches=1, num_wolves=8, num_bushes=16,
                 game_options=None, batch=1, seed=0x5EED, world_id_base=0, autoreset=True,
                 spawn_positions=None):
        from wab_gym_amd.torus_options import make_config  # config translation only

        self.cfg, self.options = make_config(width, height, num_ostriches, num_wolves, num_bushes,
                                             game_options, autoreset)
        self.B = int(batch)
        self.NO, self.NW, self.NB = int(num_ostriches), int(num_wolves), int(num_bushes)
        self.N = self.NO + self.NW + self.NB
        self.R = int(_lib().wabt_record_size(ctypes.addressof(self.cfg)))
        pos = None if spawn_positions is None else self._positions(spawn_positions)
        self.h = _lib().wabt_create_at(ctypes.addressof(self.cfg), self.B, seed, world_id_base, _p(pos))
        self.records = np.zeros((self.B, self.N, self.R), np.uint8)
        self.reward = np.zeros((self.B, self.N), np.float32)
        self.done = np.zeros((self.B, self.N), np.uint8)
        self.world_reset = np.zeros(self.B, np.uint8)

    def __del__(self):
        if getattr(self, "h", None):
            _lib().wabt_destroy(self.h)
            self.h = None

    def _positions(self, pos):
        """[N, 2] (every world alike) or [B, N, 2] int32 positions (negative: random)."""
        a = np.asarray(pos, dtype=np.int32)
        if a.shape == (self.N, 2):
            a = np.broadcast_to(a, (self.B, self.N, 2))
        if a.shape != (self.B, self.N, 2):
            raise ValueError("positions must have shape (%d, 2) or (%d, %d, 2)" % (self.N, self.B, self.N))
        return np.ascontiguousarray(a)

    def reset(self, mask=None, positions=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        pos = None if positions is None else self._positions(positions)
        _lib().wabt_reset_at(self.h, _p(m), _p(pos))

    def step(self, actions, nthreads=1):
        a = np.ascontiguousarray(actions, dtype=np.int8).reshape(self.B, self.N)
        _lib().wabt_step(self.h, _p(a), _p(self.records), _p(self.reward), _p(self.done),
                         _p(self.world_reset), int(nthreads))
        return self.records, self.reward, self.done, self.world_reset

    def state(self):
        B, N = self.B, self.N
        s = dict(df_xy=np.zeros((B, N, 2), np.int32), obj_xy=np.zeros((B, N, 2), np.int32),
                 food=np.zeros((B, N), np.float64), visible=np.zeros((B, N), np.uint8),
                 status=np.zeros((B, max(self.NO, 1)), np.uint8), turn=np.zeros(B, np.int32),
                 episode=np.zeros(B, np.uint32))
        _lib().wabt_get_state(self.h, _p(s["df_xy"]), _p(s["obj_xy"]), _p(s["food"]), _p(s["visible"]),
                              _p(s["status"]), _p(s["turn"]), _p(s["episode"]))
        return s
