import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "multihop-federeated-split-learning_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def load_pkg():
    """Import the package directory (its name is not a Python identifier) as `mhfsl_amd`."""
    if "mhfsl_amd" in sys.modules:
        return sys.modules["mhfsl_amd"]
    spec = importlib.util.spec_from_file_location("mhfsl_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mhfsl_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


@pytest.fixture(scope="session")
def fa():
    return load_pkg()


@pytest.fixture(scope="session")
def O():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def torch_gpu(fa):
    """torch on cuda:0 (import order: torch before libfa.so, they share libamdhip64)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    fa.lib()
    return torch
