"""Egocentric observation variants (wab_env.py:930-979): the oracle restatement against the
reference's own outputs (tests/golden/ego_*.npz, made by tests/golden/make_golden_ego.py)."""
import json

import numpy as np
import pytest

from oracle.oracle import OracleBatch

from golden_replay import GOLDEN_DIR

SETS = ["ego_default", "ego_wide31", "ego_sparse", "ego_empty", "ego_rect"]


def load(name):
    z = np.load("%s/%s.npz" % (GOLDEN_DIR, name))
    meta = json.loads(bytes(z["meta"]).decode())
    return z, meta


def replay_oracle(z, meta):
    """Each golden env on its own env id: autoreset-free stepping plus explicit resets, so
    the terminal observation and the reset observation are both checked."""
    ids = meta["env_ids"]
    T = meta["T"]
    for e, g in enumerate(ids):
        ob = OracleBatch(meta["options"], 1, meta["seed"], g, autoreset=False)
        _, f, r, s = ob.reset()
        assert np.array_equal(ob.egocentric()[0], z["reset0_prox"][e]), (e, "reset0")
        assert (f[0], r[0], s[0]) == tuple(z["reset0_scalars"][e])
        for t in range(T):
            _, f, r, s, rew, done = ob.step(z["actions"][t, e:e + 1])
            got = ob.egocentric()[0]
            assert np.array_equal(got, z["prox"][t, e]), (e, t, got, z["prox"][t, e])
            assert (f[0], r[0], s[0]) == tuple(z["scalars"][t, e])
            assert bool(done[0]) == bool(z["done"][t, e])
            if done[0]:
                _, f, r, s = ob.reset()
                assert np.array_equal(ob.egocentric()[0], z["rprox"][t, e]), (e, t, "reset")
                assert (f[0], r[0], s[0]) == tuple(z["rscalars"][t, e])


@pytest.mark.parametrize("name", SETS)
def test_oracle_egocentric_matches_reference_golden(name):
    z, meta = load(name)
    replay_oracle(z, meta)


def test_golden_covers_the_edge_cases():
    """The fixtures exercise: no food>0 bush in the whole seen world (all five = max_distance),
    a bush on a reachable square (= max_distance on that action), nothing in range (0)."""
    z, meta = load("ego_sparse")
    md = 11
    rows = z["prox"].reshape(-1, 5)
    assert ((rows == md).all(axis=1)).any()
    z, _ = load("ego_default")
    assert (z["prox"] == 0).any() and (z["prox"] == 11).any()
