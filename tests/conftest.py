import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


def pytest_collection_modifyitems(config, items):
    # A GPU test on a box without a GPU must fail loudly, never silently pass; but the CPU tier
    # (-m "not gpu") deselects them, so nothing to do here.
    pass
