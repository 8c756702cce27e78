"""Locate the product package (its directory name is not a Python identifier)."""
import importlib
import os
import sys

NAME = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)


def pkg():
    return importlib.import_module(NAME)


def sub(name):
    return importlib.import_module(f"{NAME}.{name}")
