"""TOOL: build variant libraries in parallel: python tools/build_variants.py [--tu FILE] name=DEF1,DEF2 name2=...
Each variant: tools/libg2048_<name>.so with the defines applied to one TU (g2048.hip by default; --tu
g2048_deep.hip for the deep kernels), the other objects shared with the shipped build."""
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: F401,E402

from rl2048_amd import _lib  # noqa: E402

_lib.build()   # the shipped library (and the shared policy object)
argv = sys.argv[1:]
tu = "g2048.hip"
if argv and argv[0] == "--tu":
    tu, argv = argv[1], argv[2:]
specs = [a.split("=", 1) for a in argv]


def one(spec):
    name, defs = spec
    d = tuple(x for x in defs.split(",") if x) if defs else ()
    return _lib.build(out=f"tools/libg2048_{name}.so", defines=d, define_tus=(tu,))


with ThreadPoolExecutor(max_workers=8) as ex:
    for r in ex.map(one, specs):
        print(r)
