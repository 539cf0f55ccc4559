"""Minimal stand-in for the ``gymnasium`` package (absent in this image, no network), used ONLY by
tests/golden/make_golden.py to import the real reference src/env.py / src/reinforce_agent.py / runner.py in the
build container.  Nothing here is on a computation path of the reference:

* ``Env.reset(seed=, options=)`` is a no-op -- real gymnasium seeds ``self.np_random`` there, which
  src/env.py never reads (its randomness is Game2048's own default_rng, src/game2048.py:102-106);
* ``spaces.Discrete(n).contains(a)`` is the only space method src/env.py calls (src/env.py:265);
  ``Box`` / ``Dict`` only record their arguments (src/env.py:79-128 builds them, nothing reads them).
"""
from . import spaces  # noqa: F401


class Env:
    metadata: dict = {}

    def __init__(self, *args, **kwargs):
        pass

    def reset(self, *, seed=None, options=None):
        return None
