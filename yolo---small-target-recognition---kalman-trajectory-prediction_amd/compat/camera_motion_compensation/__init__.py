"""Drop-in ``camera_motion_compensation`` package (reference camera_motion_compensation/):
MotionCompensatedMultiTracker.update(detections[, frame]) on the HIP tracker kernel,
MotionResetKalmanTracker (one track) and GlobalMotionDetector ('optical_flow', gmd.hip)."""
from kalman._pkg import sub

MotionCompensatedMultiTracker = sub("tracker").MotionCompensatedMultiTracker
MotionResetKalmanTracker = sub("tracker").MotionResetKalmanTracker
GlobalMotionDetector = sub("motion").GlobalMotionDetector
__all__ = ["MotionCompensatedMultiTracker", "MotionResetKalmanTracker", "GlobalMotionDetector"]
