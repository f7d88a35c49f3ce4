import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "zlib.ts_amd", "py"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libzt.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU case")


def pytest_collection_modifyitems(config, items):
    # GPU tests are only meaningful where a GPU is visible; they are selected
    # explicitly with -m gpu by the driver on the MI355X box.
    pass


@pytest.fixture(scope="session")
def oracle():
    import zt_oracle

    return zt_oracle.Oracle()
