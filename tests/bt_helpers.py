"""Synthetic detection sequences for the ByteTrack / BoT-SORT parity tests.

Targets move with constant velocity plus jitter; each frame a target is detected with a
confidence drawn from three bands (high >= 0.25, the second-association band (0.1, 0.25), and
below 0.1, which the tracker ignores), misses occur singly and in occlusion bursts (lost tracks,
re-found tracks, removal after track_buffer frames), false positives appear for a frame or two
(unconfirmed tracks that get removed), and some targets travel in tight groups (several
overlapping boxes per component of the assignment graph).  Continuous random values keep exact
cost ties away.
"""
from __future__ import annotations

import numpy as np


def scenario(seed: int, n_targets: int = 40, n_frames: int = 80, width: float = 1280.0, height: float = 720.0,
             groups: int = 4, fp_rate: float = 0.15):
    rng = np.random.default_rng(seed)
    pos = rng.uniform([60, 60], [width - 60, height - 60], (n_targets, 2))
    for g in range(groups):  # tight groups: members near a leader
        lead = rng.integers(n_targets)
        for m in rng.choice(n_targets, 3, replace=False):
            pos[m] = pos[lead] + rng.normal(0, 12, 2)
    vel = rng.normal(0, 4, (n_targets, 2))
    wh = np.c_[rng.uniform(16, 70, n_targets), rng.uniform(16, 70, n_targets)]
    occl = np.zeros(n_targets, int)
    frames = []
    for f in range(n_frames):
        pos += vel + rng.normal(0, 0.6, pos.shape)
        out = (pos[:, 0] < 0) | (pos[:, 0] > width) | (pos[:, 1] < 0) | (pos[:, 1] > height)
        vel[out] *= -1
        start = (occl == 0) & (rng.random(n_targets) < 0.02)
        occl[start] = rng.integers(2, 45, start.sum())
        seen = (occl == 0) & (rng.random(n_targets) > 0.06)
        occl = np.maximum(occl - 1, 0)
        c = pos[seen] + rng.normal(0, 1.2, (seen.sum(), 2))
        s = wh[seen] * rng.uniform(0.92, 1.08, (seen.sum(), 2))
        band = rng.random(seen.sum())
        conf = np.where(band < 0.7, rng.uniform(0.3, 0.95, seen.sum()),
                        np.where(band < 0.9, rng.uniform(0.11, 0.24, seen.sum()), rng.uniform(0.02, 0.09, seen.sum())))
        nfp = rng.poisson(fp_rate * 10)
        fc = rng.uniform([0, 0], [width, height], (nfp, 2))
        fs = rng.uniform(14, 60, (nfp, 2))
        c = np.r_[c, fc]
        s = np.r_[s, fs]
        conf = np.r_[conf, rng.uniform(0.05, 0.6, nfp)]
        order = rng.permutation(len(c))  # detector output order is arbitrary
        c, s, conf = c[order], s[order], conf[order]
        xyxy = np.c_[c - s / 2, c + s / 2].astype(np.float32)
        cls = rng.integers(0, 3, len(c)).astype(np.float32)
        frames.append((xyxy, conf.astype(np.float32), cls))
    return frames
