import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "reed-solomon_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU case")


def pytest_collection_modifyitems(config, items):
    # A GPU test on a machine without a GPU is a configuration error the -m filter should have
    # excluded; we do not silently skip it (no CPU fallback exists for the product path).
    pass
