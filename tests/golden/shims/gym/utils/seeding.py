"""gym.utils.seeding stand-in (imported, never called, by wab_env.py:4)."""
import numpy as np


def np_random(seed=None):
    rng = np.random.RandomState(seed)
    return rng, seed
