"""Import shim: ``import rl2048_amd`` loads the package directory ``rl-2048-with-reinforce-and-actor-critic_amd/``
(its name has dashes, so it cannot be imported by name).  The module replaces itself in sys.modules with the
package, so ``import rl2048_amd.agent`` etc. resolve inside that directory."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rl-2048-with-reinforce-and-actor-critic_amd")
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
