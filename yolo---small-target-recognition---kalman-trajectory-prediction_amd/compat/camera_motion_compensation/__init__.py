"""Drop-in ``camera_motion_compensation`` package (reference camera_motion_compensation/) for
the frame-free path: MotionCompensatedMultiTracker.update(detections) on the HIP tracker kernel."""
from ..kalman._pkg import sub

MotionCompensatedMultiTracker = sub("tracker").MotionCompensatedMultiTracker
__all__ = ["MotionCompensatedMultiTracker"]
