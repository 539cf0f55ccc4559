"""``gymnasium.spaces`` stand-in (see the package docstring)."""
import numpy as np


class Space:
    pass


class Discrete(Space):
    def __init__(self, n, seed=None, start=0):
        self.n = int(n)
        self.start = int(start)

    def contains(self, x) -> bool:
        # gymnasium's Discrete.contains: integer scalars (Python int or numpy integer) in [start, start + n)
        if isinstance(x, int):
            v = int(x)
        elif isinstance(x, (np.generic, np.ndarray)) and x.shape == () and np.issubdtype(x.dtype, np.integer):
            v = int(x)
        else:
            return False
        return self.start <= v < self.start + self.n


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype


class Dict(Space):
    def __init__(self, spaces=None, seed=None, **kw):
        self.spaces = dict(spaces or {}, **kw)
