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


def _batch(chance, **kw):
    opts = {"chance_wolf_on_square": chance}
    opts.update(kw)
    return orc.OracleBatch(opts, batch=1)


def test_gap_thresholds_match_c():
    for chance, margin in ((0.001, 1), (0.02, 1), (0.06, 2), (0.0, 1), (1.0, 1)):
        b = _batch(chance, wolf_spawn_margin=margin)
        T = kr.hit_threshold_lt(chance / 2)
        n = kr.GAP_CHUNK  # the oracle table (spawn sets are drawn in chunks of GAP_CHUNK tiles)
        P = kr.gap_thresholds(T, n)
        assert P[0] == 2**53 and all(P[g] >= P[g + 1] for g in range(n))
        for g in range(n + 1):
            assert P[g] == b.gap_threshold(g), (chance, g)


def test_spawn_hits_match_c():
    b = _batch(0.06)
    T = kr.hit_threshold_lt(0.03)
    P = kr.gap_thresholds(T, kr.GAP_CHUNK)
    for ep in range(40):
        ek = kr.episode_key(0x5EED, 77, ep)
        for turn in range(0, 60, 7):
            for n in (48, 121, 5, 0, 64, 65, 961):
                assert kr.spawn_hits(ek, turn, n, P) == b.spawn_hits(ek, turn, n)


def test_spawn_sets_are_iid_bernoulli():
    """The gap construction gives every tile probability q, independently: the per-index hit
    rate is flat and the set size is Binomial(n, q)."""
    q_chance = 0.2  # q = 0.1: enough hits for a tight check
    T = kr.hit_threshold_lt(q_chance / 2)
    q = T / 2**53
    n = 260  # three chunks (128, 128, 4)
    P = kr.gap_thresholds(T, kr.GAP_CHUNK)
    counts = np.zeros(n)
    sizes = []
    N = 6000
    for env in range(N):
        h = kr.spawn_hits(kr.episode_key(1, env, 0), 5, n, P)
        counts[h] += 1
        sizes.append(len(h))
    sd = np.sqrt(q * (1 - q) / N)
    assert np.all(np.abs(counts / N - q) < 5 * sd)
    sizes = np.asarray(sizes)
    assert abs(sizes.mean() - n * q) < 5 * np.sqrt(n * q * (1 - q) / N)
    assert abs(sizes.var() - n * q * (1 - q)) < 0.15 * n * q * (1 - q)
    # pairwise independence of two fixed tiles
    both = 0
    for env in range(N):
        h = set(kr.spawn_hits(kr.episode_key(1, env, 0), 5, n, P))
        both += (3 in h) and (40 in h)
    assert abs(both / N - q * q) < 5 * np.sqrt(q * q / N)


def test_conditional_spawn_U_sides():
    T = kr.hit_threshold_lt(0.0005)
    rng = np.random.RandomState(3)
    for V in list(rng.randint(0, 2**53, size=200, dtype=np.int64)) + [0, 2**53 - 1]:
        lo = kr.conditional_spawn_U(int(V), T, True)
        hi = kr.conditional_spawn_U(int(V), T, False)
        assert 0 <= lo < T <= hi < 2**53
        assert (lo * 2.0**-53 < 0.0005) and not (hi * 2.0**-53 < 0.0005)


def test_ring_and_view_index_are_bijections():
    for W, H, m in ((11, 11, 1), (13, 11, 2), (31, 31, 1), (3, 5, 3)):
        cw, ch = W // 2, H // 2
        ring = [kr.ring_index(dx, dy, W, H, m) for dx in range(-cw - m, cw + m + 1)
                for dy in range(-ch - m, ch + m + 1) if abs(dx) > cw or abs(dy) > ch]
        assert sorted(ring) == list(range((W + 2 * m) * (H + 2 * m) - W * H))
        view = [kr.view_index(dx, dy, W, H) for dx in range(-cw, cw + 1) for dy in range(-ch, ch + 1)]
        assert sorted(view) == list(range(W * H))
