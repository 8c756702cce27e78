"""kalman.trajectory_visualizer stand-in.

The reference's visualizer (kalman/trajectory_visualizer.py) is cv2 drawing and is outside
the hot path.  This pass-through keeps the driver's import and call
working: draw_tracks returns the frame unchanged."""


class TrajectoryVisualizer:
    def __init__(self, *args, **kwargs):
        pass

    def draw_tracks(self, frame, tracks, detections=None, frame_info=None):
        return frame
