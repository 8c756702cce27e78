"""Synthetic detection sequences that exercise the motion-reset tracker's three reset triggers
(position jumps, velocity changes, size changes), occlusions and re-appearances.  Detections
are lists of [x1, y1, x2, y2, conf] with np.float32 elements, as the reference driver builds
them (aircraft_detection_tracking.py:99-106)."""
import numpy as np


def jumpy_sequence(seed: int, K: int = 12, T: int = 160, W: int = 640, H: int = 512, events: bool = True,
                   dup: float = 0.0, shuffle: bool = True):
    """dup: probability that a visible target also yields a second box shifted by 2-8 px (the
    planted detector's two-boxes-per-target clutter): the association rounds then hold chains
    of overlapping candidates, and pairs of already matched rows and columns stay candidates
    in later rounds.  shuffle=False lists the targets in index order (a duplicate right after its
    box), so detection 0 and the oldest track (list position 0) overlap on most frames."""
    rng = np.random.default_rng(seed)
    pos = rng.uniform([40, 40], [W - 40, H - 40], (K, 2))
    vel = rng.uniform(-2.0, 2.0, (K, 2))
    size = rng.uniform([8, 6], [24, 18], (K, 2))
    hidden = np.zeros(K, dtype=int)
    frames = []
    for t in range(T):
        pos += vel
        for k in range(K):
            for j, lim in enumerate((W, H)):
                if pos[k, j] < 20 or pos[k, j] > lim - 20:
                    vel[k, j] = -vel[k, j]
        if events and t > 5:
            for k in range(K):
                u = rng.uniform()
                if u < 0.015:      # camera shake / re-detection elsewhere: a jump of 45-90 px
                    pos[k] += rng.choice([-1, 1], 2) * rng.uniform(45, 90, 2)
                    pos[k] = np.clip(pos[k], 25, [W - 25, H - 25])
                elif u < 0.03:     # size change of 35-60 %
                    size[k] *= rng.choice([0.55, 1.6])
                    size[k] = np.clip(size[k], 4, 48)
                elif u < 0.04:     # sudden velocity change
                    vel[k] = rng.uniform(-6, 6, 2)
                elif u < 0.05:     # occlusion burst
                    hidden[k] = int(rng.integers(1, 25))
        dets = []
        order = rng.permutation(K) if shuffle else np.arange(K)
        for k in order:
            if hidden[k] > 0:
                hidden[k] -= 1
                continue
            c = pos[k] + rng.normal(0, 0.4, 2)
            w, h = size[k] * rng.uniform(0.95, 1.05, 2)
            b = np.array([c[0] - w / 2, c[1] - h / 2, c[0] + w / 2, c[1] + h / 2], np.float32)
            dets.append([b[0], b[1], b[2], b[3], np.float32(rng.uniform(0.3, 0.95))])
            if dup and rng.uniform() < dup:
                o = (rng.choice([-1, 1], 2) * rng.uniform(2, 8, 2)).astype(np.float32)
                dets.append([b[0] + o[0], b[1] + o[1], b[2] + o[0], b[3] + o[1], np.float32(rng.uniform(0.3, 0.95))])
        frames.append(dets)
    return frames
