"""Drop-in ``ultralytics`` package exposing ``YOLO`` for the detection predict path
(ultralytics/__init__.py, engine/model.py) backed by libyk.so."""
from ._pkg import sub

_p = sub("predictor")
YOLO = _p.YOLO
Results = _p.Results
Boxes = _p.Boxes
__version__ = "8.3.193"
__all__ = ["YOLO"]
