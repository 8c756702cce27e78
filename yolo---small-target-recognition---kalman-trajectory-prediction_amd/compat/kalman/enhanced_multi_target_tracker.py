"""kalman.enhanced_multi_target_tracker -> HIP tracker (see package tracker.py)."""
from ._pkg import sub

_t = sub("tracker")
EnhancedMultiTargetTracker = _t.EnhancedMultiTargetTracker
AircraftKalmanTracker = _t.AircraftKalmanTracker
