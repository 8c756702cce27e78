"""camera_motion_compensation.global_motion_detector -> GlobalMotionDetector on the gmd.hip
kernels (global_motion_detector.py:11-288; 'optical_flow' only)."""
from kalman._pkg import sub

GlobalMotionDetector = sub("motion").GlobalMotionDetector
