import os
import sys

import pytest

try:  # load torch's HIP runtime before libmpgpu so device pointers and streams are shared
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmpgpu on cuda:0)")
    lib = os.path.join(ROOT, "motionplanning_amd", "lib", "libmpgpu.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        import __graft_entry__

        __graft_entry__.build()


@pytest.fixture(scope="session")
def ctx():
    from motionplanning_amd.context import default_context

    return default_context(0)
