"""gym 0.17.2 `spaces` subset used by the reference (Discrete / Box / Tuple + flatdim/flatten).

flatten/flatdim follow gym 0.17.2's published semantics: Discrete(n) -> one-hot of
length n, Box -> ravel (float), Tuple -> concatenation in order.  gym's own source is
not available offline, so the C5 featurizer layout built on it is "parity unpinned".
"""
import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = shape
        self.dtype = None if dtype is None else np.dtype(dtype)


class Discrete(Space):
    def __init__(self, n):
        self.n = int(n)
        super().__init__((), np.int64)

    def sample(self):
        return int(np.random.randint(self.n))

    def __repr__(self):
        return "Discrete(%d)" % self.n


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        super().__init__(tuple(shape) if shape is not None else np.shape(low), dtype)
        self.low = low
        self.high = high

    def __repr__(self):
        return "Box%s" % (self.shape,)


class Tuple(Space):
    def __init__(self, spaces):
        self.spaces = tuple(spaces)
        super().__init__(None, None)

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)


def flatdim(space):
    if isinstance(space, Box):
        return int(np.prod(space.shape))
    if isinstance(space, Discrete):
        return space.n
    if isinstance(space, Tuple):
        return int(sum(flatdim(s) for s in space.spaces))
    raise NotImplementedError(type(space))


def flatten(space, x):
    if isinstance(space, Box):
        return np.asarray(x, dtype=space.dtype).flatten()
    if isinstance(space, Discrete):
        onehot = np.zeros(space.n, dtype=np.float32)
        onehot[x] = 1.0
        return onehot
    if isinstance(space, Tuple):
        return np.concatenate([flatten(s, x_part) for x_part, s in zip(x, space.spaces)])
    raise NotImplementedError(type(space))
