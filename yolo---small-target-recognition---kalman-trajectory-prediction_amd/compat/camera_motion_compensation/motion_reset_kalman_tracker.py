"""camera_motion_compensation.motion_reset_kalman_tracker -> one motion-reset track on the HIP
tracker (motion_reset_kalman_tracker.py:16-355: update / predict / get_track_info /
get_reset_statistics)."""
from kalman._pkg import sub

MotionResetKalmanTracker = sub("tracker").MotionResetKalmanTracker
