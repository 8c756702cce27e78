import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_NAME = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the built libyk.so")
    config.addinivalue_line("markers", "slow: long-running")


def pkg():
    return importlib.import_module(PKG_NAME)


@pytest.fixture(scope="session")
def yk():
    return pkg()
