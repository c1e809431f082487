"""The step kernels' bush value (generate_n_bush_values, wab_env.py:631-635) is the exact
count of thresholds T_k <= U (tests/test_thresholds.py pins the table against the
reference's numpy expression).  The kernels find it with a float guess bracketed by four
table entries (bush_value_fast, wab_device.h); here the device result is compared with the
CPU count on every threshold boundary +-64 and on millions of random draws, for the default
options and for other powers/maxima (where the guess misses more often and the exact
fallback has to take over)."""
import ctypes

import numpy as np
import pytest

from wab_gym_amd import _lib

pytestmark = pytest.mark.gpu


def device_values(env, U):
    import torch

    u = torch.as_tensor(U.astype(np.uint64).view(np.int64), device=env.device)
    out = torch.empty(len(U), dtype=torch.int32, device=env.device)
    _lib.check(_lib.load().wab_debug_bush_values(env._h, u.data_ptr(), out.data_ptr(), len(U),
                                                 ctypes.c_void_p(torch.cuda.current_stream(env.device).cuda_stream)),
               "wab_debug_bush_values")
    torch.cuda.synchronize(env.device)
    return out.cpu().numpy()


@pytest.mark.parametrize("opts", [{}, {"bush_power": 2.5, "max_berries_per_bush": 7},
                                  {"bush_power": 1, "max_berries_per_bush": 255},
                                  {"bush_power": 400, "max_berries_per_bush": 50}])
def test_bush_value_matches_threshold_count(opts):
    from wab_gym_amd.env import BatchedWolvesAndBushesEnv
    from wab_gym_amd.options import bush_thresholds, default_game_options

    o = dict(default_game_options, **opts)
    thr = bush_thresholds(o["bush_power"], o["max_berries_per_bush"]).astype(np.uint64)
    env = BatchedWolvesAndBushesEnv(opts, num_envs=64, device="cuda:0")
    rng = np.random.default_rng(7)
    d = np.arange(-64, 65, dtype=np.int64)
    edges = (thr[:, None].astype(np.int64) + d[None, :]).ravel()
    U = np.concatenate([
        edges[(edges >= 0) & (edges < (1 << 53))].astype(np.uint64),
        rng.integers(0, 1 << 53, size=2_000_000, dtype=np.uint64),
        # the top of the range, where the large values live
        ((1 << 53) - 1 - rng.integers(0, 1 << 40, size=500_000, dtype=np.uint64)).astype(np.uint64),
        np.array([0, 1, (1 << 53) - 1], dtype=np.uint64),
    ])
    want = np.searchsorted(thr, U, side="right").astype(np.int32)
    got = device_values(env, U)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (U[bad[:5]], got[bad[:5]], want[bad[:5]])
