"""Shared pytest setup: the `gpu` marker, repo root on sys.path, and torch imported before any HIP library.

torch ships its own libamdhip64.so (SONAME libamdhip64.so.7); importing torch first makes the dynamic linker
resolve the product library's libamdhip64 dependency to that same runtime, so both share one HIP context.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (see module docstring)

# tools/ab_grad.sh only: run the parity tests against another build of libg2048 (the shipped library otherwise)
if os.environ.get("G2048_TOOLS_LIB"):
    from rl2048_amd import _lib as _L

    _L.use_library_for_tools(os.environ["G2048_TOOLS_LIB"])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


def gpu_available() -> bool:
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
