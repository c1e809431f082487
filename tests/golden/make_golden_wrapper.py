"""Golden vectors for the device featurizers: the reference `PragmaticObsWrapper.observation`
(wab_env.py:726-824) and `SuperBasicObservationWrapper.observation` (:900-927), each followed
by gym 0.17's `spaces.flatten` (actor_critic.py:188).

Container-only (imports /root/reference through ref_harness).  Inputs are random wolf/bush
grids of several densities plus the three hand-built grids of the reference's own KATs
(wab_env_test.py:9-169); outputs are the wrappers' tuples flattened to float32 ([449] and [90] at 11x11).
`flatten` is restated by the gym stub (gym is not installed): that layout is "parity
unpinned" (SURVEY.md §8c); the wrapper's values themselves are pinned by the reference.

Usage: python tests/golden/make_golden_wrapper.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness as rh  # noqa: E402


def kat_inputs():
    """The three grids built by wab_env_test.py (data only; see that file for provenance)."""
    out = []
    w, b = np.zeros((11, 11)), np.zeros((11, 11))
    b[6, 3] = b[7, 4] = b[8, 6] = b[6, 10] = 1
    w[5, 5] = w[6, 6] = w[4, 4] = 1
    out.append((w, b))
    w, b = np.zeros((11, 11)), np.zeros((11, 11))
    b[5, 5] = 1
    out.append((w, b))
    from wab_gym_amd.options import LOOKOUT_MASK

    w, b = np.zeros((11, 11)), np.zeros((11, 11))
    w[2, :] = 1
    w[:, 6] = 1
    b[1, :] = 1
    b[9, :] = 1
    w[np.where(LOOKOUT_MASK == 1)] = 0
    b[np.where(LOOKOUT_MASK == 1)] = 0
    out.append((w, b))
    return out


def main():
    import gym  # the stub

    wab_env = rh.load_reference()
    env = rh.make_env(0x5EED, 0)
    wrapper = wab_env.PragmaticObsWrapper(env)
    space = wrapper.observation_space
    from wab_gym_amd.options import LOOKOUT_MASK, GATHERER_MASK

    rng = np.random.RandomState(7)
    grids, scal, masks = [], [], []
    for w, b in kat_inputs():
        grids.append(np.stack([w, b, np.zeros((11, 11))]))
        scal.append((40, 0, 0))
        masks.append(LOOKOUT_MASK)
    for n in range(1500):
        dw = rng.choice([0.0, 0.005, 0.02, 0.1, 0.5])
        db = rng.choice([0.0, 0.01, 0.06, 0.2, 0.6, 1.0])
        w = (rng.random_sample((11, 11)) < dw).astype(float)
        b = (rng.random_sample((11, 11)) < db).astype(float)
        o = np.zeros((11, 11))
        o[5, 5] = 1
        grids.append(np.stack([w, b, o]))
        scal.append((rng.randint(41), rng.randint(2), rng.randint(3)))
        masks.append([np.zeros((11, 11)), LOOKOUT_MASK, GATHERER_MASK][rng.randint(3)])
    feats, sb_feats, sb_raw = [], [], []
    superbasic = wab_env.SuperBasicObservationWrapper(env)
    sb_space = superbasic.observation_space
    for g, (f, r, s), m in zip(grids, scal, masks):
        obs = (g[0], g[1], g[2], f, r, s, m)
        feats.append(gym.spaces.flatten(space, wrapper.observation(obs)))
        sb = superbasic.observation(obs)
        sb_raw.append(list(sb[0]) + [sb[1], sb[2], sb[3]])
        sb_feats.append(gym.spaces.flatten(sb_space, sb))
    out = {
        "planes": np.stack(grids).astype(np.uint8),
        "scalars": np.asarray(scal, dtype=np.uint8),
        "view_mask": np.stack(masks).astype(np.uint8),
        "features": np.stack(feats).astype(np.float32),
        "flatdim": np.int64(gym.spaces.flatdim(space)),
    }
    np.savez_compressed(os.path.join(HERE, "pragmatic.npz"), **out)
    print("pragmatic.npz: %d cases, flatdim %d" % (len(feats), out["flatdim"]))
    sb_out = {
        "planes": out["planes"],
        "scalars": out["scalars"],
        "raw": np.asarray(sb_raw, dtype=np.int32),  # nearest_bush[4], food, role, status
        "features": np.stack(sb_feats).astype(np.float32),
        "flatdim": np.int64(gym.spaces.flatdim(sb_space)),
    }
    np.savez_compressed(os.path.join(HERE, "superbasic.npz"), **sb_out)
    print("superbasic.npz: %d cases, flatdim %d" % (len(sb_feats), sb_out["flatdim"]))


if __name__ == "__main__":
    main()
