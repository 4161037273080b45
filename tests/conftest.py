import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def O():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def ob():
    return importlib.import_module("oaxaca-blinder-rs_amd")


@pytest.fixture(scope="session")
def N(ob):
    return ob._native
