"""The numpy keyed-RNG twin (oracle/keyed_rng.py) and the C oracle agree on every draw."""
import numpy as np

from oracle import keyed_rng as kr
from oracle import oracle as orc


def test_episode_key_matches_c():
    rng = np.random.RandomState(0)
    for _ in range(200):
        seed, env, ep = (int(v) for v in rng.randint(0, 2**62, size=3, dtype=np.int64))
        assert kr.episode_key(seed, env, ep) == orc.episode_key(seed, env, ep)


def test_draws_match_c():
    rng = np.random.RandomState(1)
    ek = kr.episode_key(0x5EED, 12345, 7)
    x = rng.randint(-40000, 40000, size=500)
    y = rng.randint(-40000, 40000, size=500)
    turn = rng.randint(0, 2**21, size=500)
    k = rng.randint(0, 300, size=500)
    for site in (1, 2, 3, 4, 5, 9):
        U = kr.draw_U(ek, site, turn, x, y, k)
        for i in range(0, 500, 7):
            assert int(U[i]) == orc.draw_U(ek, site, int(turn[i]), int(x[i]), int(y[i]), int(k[i]))
        assert (U < 2**53).all()


def test_draws_look_uniform():
    ek = kr.episode_key(0x5EED, 3, 0)
    xs, ys = np.meshgrid(np.arange(-200, 200), np.arange(-200, 200))
    u = kr.draw_u(ek, kr.SITE_BUSH, 0, xs.ravel(), ys.ravel())
    assert abs(u.mean() - 0.5) < 0.005
    hist = np.histogram(u, bins=20, range=(0, 1))[0]
    assert hist.min() > 0.9 * len(u) / 20


def test_integer_thresholds_equal_float_compares():
    rng = np.random.RandomState(2)
    for p in (0.05, 0.0005, 0.001 / 2, 0.2, 1e-9, 0.5):
        keep = kr.keep_threshold_gt(p)
        hit = kr.hit_threshold_lt(p)
        U = np.concatenate([rng.randint(0, 2**53, size=1000, dtype=np.int64),
                            np.arange(keep - 3, keep + 4), np.arange(hit - 3, hit + 4)])
        U = U[(U >= 0) & (U < 2**53)]
        u = U.astype(np.float64) * 2.0**-53
        assert np.array_equal(U > keep, u > p)
        assert np.array_equal(U < hit, u < p)
