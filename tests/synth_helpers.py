"""Scene helpers shared by CPU and GPU tests."""
from conftest import pkg


def scene_dets(seed=0, n_targets=16, n_frames=50, **kw):
    """GT-injected float32 detections of a synthetic scene, one list per frame."""
    sc = pkg().synth.Scene(seed=seed, n_targets=n_targets, n_frames=n_frames, **kw)
    return [sc.detections(t) for t in range(n_frames)]
