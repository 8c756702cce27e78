"""kalman.enhanced_aircraft_kalman_tracker -> HIP single-track object (see package tracker.py)."""
from ._pkg import sub

_t = sub("tracker")
AircraftKalmanTracker = _t.AircraftKalmanTracker
EnhancedAircraftKalmanTracker = AircraftKalmanTracker
