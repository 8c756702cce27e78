"""camera_motion_compensation.motion_compensated_multi_tracker -> HIP tracker (motion-reset policy)."""
from kalman._pkg import sub

MotionCompensatedMultiTracker = sub("tracker").MotionCompensatedMultiTracker
