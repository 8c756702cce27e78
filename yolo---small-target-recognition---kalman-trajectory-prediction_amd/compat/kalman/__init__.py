"""Drop-in ``kalman`` package (reference kalman/__init__.py:28-45) backed by libyk.so.

Put ``<repo>/yolo---small-target-recognition---kalman-trajectory-prediction_amd/compat`` on
sys.path and ``from kalman.enhanced_multi_target_tracker import EnhancedMultiTargetTracker``
(kalman/aircraft_detection_tracking.py:26) resolves to the HIP tracker.
"""
from ._pkg import sub

_t = sub("tracker")
EnhancedAircraftKalmanTracker = _t.AircraftKalmanTracker
EnhancedMultiTargetTracker = _t.EnhancedMultiTargetTracker
AircraftKalmanTracker = EnhancedAircraftKalmanTracker
MultiTargetTracker = EnhancedMultiTargetTracker

__all__ = ["AircraftKalmanTracker", "EnhancedAircraftKalmanTracker", "EnhancedMultiTargetTracker",
           "MultiTargetTracker"]
__version__ = "2.0.0"
