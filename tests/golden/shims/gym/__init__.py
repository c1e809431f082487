"""Minimal offline stand-in for gym 0.17.2 (container-only golden-vector harness).

gym is not installed and cannot be fetched (no network).  The reference's
`wab_env.py` imports only a handful of names from it (`wab_env.py:1-4`); this
stub provides exactly those, with gym 0.17 semantics where they matter:
`Env.seed` is a no-op (gym 0.17's base class), wrappers delegate unknown
attributes to the wrapped env (`PragmaticObsWrapper.__init__` reads
`self.game_options`, `wab_env.py:709`).

Never shipped as product code; only `tests/golden/make_golden.py` and the CPU
test-suite's reference-KAT check put this directory on `sys.path`.
"""
from . import spaces, logger, wrappers  # noqa: F401
from .utils import seeding  # noqa: F401


class Env:
    metadata = {"render.modes": []}
    spec = None

    def seed(self, seed=None):  # gym 0.17 base class: no-op
        return None

    def close(self):
        return None


class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self.action_space = getattr(env, "action_space", None)
        self.observation_space = getattr(env, "observation_space", None)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        return self.env.step(action)


class ObservationWrapper(Wrapper):
    def reset(self, **kwargs):
        return self.observation(self.env.reset(**kwargs))

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        return self.observation(obs), reward, done, info

    def observation(self, observation):
        raise NotImplementedError
