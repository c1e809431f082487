"""Minimal gym-style space descriptors (gym itself is not a dependency).

They carry the same shapes and sizes as the reference's spaces
(`initialize_action_space` / `initialize_observation_space`, wab_env.py:188-229).
"""
from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def sample(self, size=None, generator=None, device=None):
        import torch

        shape = () if size is None else (size if isinstance(size, tuple) else (int(size),))
        return torch.randint(0, self.n, shape, generator=generator, device=device, dtype=torch.int64)

    def contains(self, x):
        return 0 <= int(x) < self.n

    def __repr__(self):
        return "Discrete(%d)" % self.n


class Box:
    def __init__(self, low, high, shape, dtype=np.uint8):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

    def __repr__(self):
        return "Box(%s, %s, %s, %s)" % (self.low, self.high, self.shape, self.dtype)


class Tuple:
    def __init__(self, spaces):
        self.spaces = tuple(spaces)

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)

    def __repr__(self):
        return "Tuple(%s)" % ", ".join(map(repr, self.spaces))


class DummySpec:
    """Mirror of the reference's DummySpec (wab_env.py:87-100)."""

    def __init__(self, id, reward_threshold=None, nondeterministic=False, max_episode_steps=None,
                 kwargs=None):
        self.id = id
        self.reward_threshold = reward_threshold
        self.nondeterministic = nondeterministic
        self.max_episode_steps = max_episode_steps
