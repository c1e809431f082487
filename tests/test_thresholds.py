"""The bush threshold table reproduces `np.round(u ** power * max)` (wab_env.py:632-635)."""
import numpy as np
import pytest

from wab_gym_amd.options import bush_thresholds


def _value(U, power, mx):
    u = np.asarray(U, dtype=np.int64).astype(np.float64) * 2.0**-53
    return np.round(u ** power * mx)


def _lookup(T, U):
    return np.searchsorted(T, np.asarray(U, dtype=np.uint64), side="right")


@pytest.mark.parametrize("power,mx", [(100, 200), (60, 200), (100, 255), (2.5, 7), (1, 1)])
def test_every_boundary(power, mx):
    T = bush_thresholds(power, mx).astype(np.int64)
    assert np.all(np.diff(T) >= 0)
    for k, t in enumerate(T, start=1):
        if t >= 2**53:
            continue
        around = np.arange(max(t - 64, 0), min(t + 64, 2**53))
        assert np.array_equal(_lookup(T, around), _value(around, power, mx).astype(np.int64)), k


def test_random_draws_default():
    rng = np.random.RandomState(5)
    T = bush_thresholds(100, 200)
    lo = int(T[0]) - 2**40
    U = np.concatenate([rng.randint(0, 2**53, size=200000, dtype=np.int64),
                        rng.randint(lo, 2**53, size=200000, dtype=np.int64)])
    assert np.array_equal(_lookup(T, U), _value(U, 100, 200).astype(np.int64))


def test_presence_probability():
    T = bush_thresholds(100, 200)
    p = 1 - T[0] / 2.0**53
    assert abs(p - (1 - 0.0025 ** 0.01)) < 1e-6   # P(food > 0) = 0.0582
