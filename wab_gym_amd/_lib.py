"""ctypes binding of the C-ABI in include/wab.h (libwab_hip.so, built in-tree).

There is no fallback: if the HIP library is missing or fails to load, every product
entry point raises.  torch is imported first so that its bundled HIP runtime
(SONAME libamdhip64.so.7) is the one the library binds to — one runtime per process.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WAB_LIB") or os.path.join(HERE, "_lib", "libwab_hip.so")

EXPORTED = [
    "wab_abi_version", "wab_last_error", "wab_num_actions", "wab_create", "wab_destroy",
    "wab_reset", "wab_step", "wab_rollout", "wab_get_counters", "wab_get_state", "wab_batch",
    "wab_feature_dim", "wab_featurize", "wab_discounted_returns", "wab_step_kernel",
    "wab_superbasic_dim", "wab_featurize_superbasic", "wab_render", "wab_egocentric",
    "wab_debug_bush_values", "wab_step_features", "wab_discounted_returns_exact",
    "wab_bush_thresholds", "wab_rollout_features", "wab_render_envs", "wab_set_obs_placement",
    # include/wab_torus.h: the Environment 2.0 torus world
    "wab2_abi_version", "wab2_last_error", "wab2_record_size", "wab2_create", "wab2_destroy",
    "wab2_batch", "wab2_reset", "wab2_step", "wab2_rollout", "wab2_get_state", "wab2_get_counters",
    "wab2_get_obs", "wab2_take_action", "wab2_create_at", "wab2_reset_at",
]

ABI2_VERSION = 1
OBS_SAME_BUFFER, OBS_FRESH_BUFFER = 0, 1  # wab_set_obs_placement

ABI_VERSION = 5


class WabObs(ctypes.Structure):
    _fields_ = [("planes", ctypes.c_void_p), ("food_turns", ctypes.c_void_p),
                ("role", ctypes.c_void_p), ("status", ctypes.c_void_p)]


class WabCounters(ctypes.Structure):
    _fields_ = [("wolf_overflow", ctypes.c_uint64), ("eaten_overflow", ctypes.c_uint64),
                ("bad_actions", ctypes.c_uint64), ("steps", ctypes.c_uint64),
                ("resets", ctypes.c_uint64), ("ego_missing", ctypes.c_uint64),
                ("handoff_timeouts", ctypes.c_uint64), ("wolf_overflow_reset", ctypes.c_uint64),
                ("rollout_launches", ctypes.c_uint64), ("rollout_step_calls", ctypes.c_uint64)]


class WabError(RuntimeError):
    pass


_lib = None


def load():
    """Load libwab_hip.so (raises if it is absent: build it with __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WabError("libwab_hip.so not built (%s); run `python -c 'import __graft_entry__ as g; "
                       "g.build()'`" % LIB_PATH)
    try:
        import torch  # noqa: F401  (bind to torch's HIP runtime if torch is used)
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    if hasattr(L, "wab_diagnostic_build") and os.environ.get("WAB_DIAGNOSTIC_OK") != "1":
        # a stamps / store-floor / ablation build (csrc/wab_build_guard.h): results wrong by design
        raise WabError("%s is a diagnostic build (wab_diagnostic_build); the product library is "
                       "wab_gym_amd/_lib/libwab_hip.so (set WAB_DIAGNOSTIC_OK=1 only in tools/)" % LIB_PATH)
    P, I64, U64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32
    L.wab_abi_version.restype = ctypes.c_int
    L.wab_last_error.restype = ctypes.c_char_p
    L.wab_num_actions.argtypes = [P]
    L.wab_create.argtypes = [P, I64, U64, I64, ctypes.c_int, ctypes.POINTER(P)]
    L.wab_destroy.argtypes = [P]
    L.wab_reset.argtypes = [P, P, P, P]
    L.wab_step.argtypes = [P, P, P, P, P, P, P]
    L.wab_rollout.argtypes = [P, P, I32, P, P, P, P]
    L.wab_get_counters.argtypes = [P, P, P]
    L.wab_get_state.argtypes = [P, P, P, P, P, P, P, P]
    L.wab_feature_dim.argtypes = [P]
    L.wab_featurize.argtypes = [P, P, P, P, P]
    L.wab_superbasic_dim.argtypes = [P]
    L.wab_featurize_superbasic.argtypes = [P, P, P, P]
    L.wab_step_features.argtypes = [P, P, P, P, P, P, P]
    L.wab_render.argtypes = [P, P, I32, I32, P, P]
    L.wab_render_envs.argtypes = [P, P, I64, I64, I32, I32, P, P]
    L.wab_egocentric.argtypes = [P, P, P, P]
    L.wab_debug_bush_values.argtypes = [P, P, P, I64, P]
    L.wab_discounted_returns.argtypes = [P, P, I32, I64, ctypes.c_double, P, P, P]
    L.wab_discounted_returns_exact.argtypes = [P, P, P, I32, I64, ctypes.c_double, P, P, P]
    L.wab_bush_thresholds.argtypes = [ctypes.c_double, I32, P]
    L.wab_rollout_features.argtypes = [P, P, I32, P, P, P, P, ctypes.c_double, P, P, P]
    L.wab_batch.argtypes = [P]
    L.wab_batch.restype = I64
    L.wab_step_kernel.argtypes = [P]
    L.wab_step_kernel.restype = ctypes.c_char_p
    L.wab_set_obs_placement.argtypes = [P, I32]
    L.wab2_abi_version.restype = ctypes.c_int
    L.wab2_last_error.restype = ctypes.c_char_p
    L.wab2_record_size.argtypes = [P]
    L.wab2_create.argtypes = [P, I64, U64, I64, ctypes.c_int, ctypes.POINTER(P)]
    L.wab2_destroy.argtypes = [P]
    L.wab2_batch.argtypes = [P]
    L.wab2_batch.restype = I64
    L.wab2_reset.argtypes = [P, P, P]
    L.wab2_create_at.argtypes = [P, I64, U64, I64, ctypes.c_int, P, ctypes.POINTER(P)]
    L.wab2_reset_at.argtypes = [P, P, P, P]
    L.wab2_step.argtypes = [P, P, P, P, P, P, P]
    L.wab2_rollout.argtypes = [P, P, I32, P, P, P, P, P]
    L.wab2_get_state.argtypes = [P] * 9
    L.wab2_get_counters.argtypes = [P, P, P]
    L.wab2_get_obs.argtypes = [P, I32, P, P]
    L.wab2_take_action.argtypes = [P, I32, P, P, P, P, P]
    for name in EXPORTED:
        if name not in ("wab_abi_version", "wab_last_error", "wab_batch", "wab_step_kernel",
                        "wab2_abi_version", "wab2_last_error", "wab2_batch"):
            getattr(L, name).restype = ctypes.c_int
    if L.wab_abi_version() != ABI_VERSION:
        raise WabError("libwab_hip.so ABI %d != %d" % (L.wab_abi_version(), ABI_VERSION))
    if L.wab2_abi_version() != ABI2_VERSION:
        raise WabError("libwab_hip.so torus ABI %d != %d" % (L.wab2_abi_version(), ABI2_VERSION))
    _lib = L
    return L


class Wab2Counters(ctypes.Structure):
    _fields_ = [("turns", ctypes.c_uint64), ("resets", ctypes.c_uint64)]


def check2(rc, what="wab2 call"):
    """check() for the torus entry points (their own wab2_last_error)."""
    if rc != 0:
        msg = load().wab2_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError("%s: %s" % (what, msg))
        raise WabError("%s failed (%d): %s" % (what, rc, msg))


def check(rc, what="wab call"):
    if rc != 0:
        msg = load().wab_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError("%s: %s" % (what, msg))
        raise WabError("%s failed (%d): %s" % (what, rc, msg))
