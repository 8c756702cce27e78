"""MI355X-native detect-and-track hot path (YOLOv8-small+P2 predict -> Kalman tracker).

Drop-in for the two Python surfaces of the reference's per-frame loop
(kalman/aircraft_detection_tracking.py:88-131):
  * ``YOLO(...)(frame)``                    -> ultralytics.YOLO.predict (engine/model.py:498-557)
  * ``EnhancedMultiTargetTracker.update``   -> kalman/enhanced_multi_target_tracker.py:42-132
Both execute in libyk.so (hand-written HIP for gfx950, C ABI in include/yk.h).  There is no
CPU fallback: without the library or a GPU every entry point raises ``YKError``.

``compat/`` holds ``kalman`` and ``ultralytics`` shim packages: put that directory on
sys.path and the reference driver's imports resolve to this package unchanged.
"""
from . import arch, frames, model, predictor, shard, synth, tracker, visualize, weights  # noqa: F401
from ._lib import YKError, exported_symbols  # noqa: F401
from .tracker import (  # noqa: F401
    AircraftKalmanTracker,
    EnhancedAircraftKalmanTracker,
    EnhancedMultiTargetTracker,
    MotionCompensatedMultiTracker,
    MotionResetKalmanTracker,
    MultiStreamTracker,
    MultiTargetTracker,
)
from .predictor import YOLO, Boxes, Results  # noqa: F401
from .visualize import TrajectoryVisualizer  # noqa: F401

__version__ = "0.1.0"
