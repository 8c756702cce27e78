"""kalman.trajectory_visualizer (reference kalman/trajectory_visualizer.py:5-235).

Resolves to the package's host-side visualizer (visualize.py): the same colours, labels,
flashing predicted boxes with the 0.3 / 0.7 fill, trails and velocity arrows, drawn on numpy
BGR frames with restated OpenCV primitives (cv2 is not in this image)."""
from ._pkg import sub

TrajectoryVisualizer = sub("visualize").TrajectoryVisualizer

__all__ = ["TrajectoryVisualizer"]
