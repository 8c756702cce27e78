"""Synthetic camera-pan sequences for the global camera-motion detector tests.

A textured "world" (smoothed noise, rectangles, discs) is viewed through a moving camera: each
frame is a bilinear resample of the world at a (fractional) camera offset, plus a few small
bright targets moving on their own and mild sensor noise.  Offsets come from a scripted path
(steady pan, a fast whip pan that must trigger a reset, a still stretch), so the detector's
branches -- no motion, motion, reset, motion consistency -- are all exercised.
"""
from __future__ import annotations

import numpy as np


def _smooth_noise(rng, h, w, cell):
    base = rng.normal(0, 1, (h // cell + 3, w // cell + 3))
    ys = np.arange(h) / cell
    xs = np.arange(w) / cell
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    return (base[y0][:, x0] * (1 - fy) * (1 - fx) + base[y0][:, x0 + 1] * (1 - fy) * fx +
            base[y0 + 1][:, x0] * fy * (1 - fx) + base[y0 + 1][:, x0 + 1] * fy * fx)


def make_world(seed: int, h: int, w: int) -> np.ndarray:
    """Structure at several scales (coarse pyramid levels need texture too): smooth noise at
    40 px and 10 px cells, rectangles and discs of 8-60 px, fine sensor-like noise."""
    rng = np.random.default_rng(seed)
    img = 115 + 40 * _smooth_noise(rng, h, w, 40) + 14 * _smooth_noise(rng, h, w, 10) + rng.normal(0, 4, (h, w))
    for _ in range(h * w // 2500):  # rectangles: strong corners
        y, x = rng.integers(0, h - 60), rng.integers(0, w - 60)
        img[y:y + rng.integers(8, 60), x:x + rng.integers(8, 60)] += rng.uniform(-60, 60)
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(h * w // 15000):  # discs
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(4, 25)
        img[(yy - cy) ** 2 + (xx - cx) ** 2 < r * r] += rng.uniform(-50, 50)
    return np.clip(img, 0, 255)


def _sample(world: np.ndarray, oy: float, ox: float, h: int, w: int) -> np.ndarray:
    y0, x0 = int(np.floor(oy)), int(np.floor(ox))
    fy, fx = oy - y0, ox - x0
    a = world[y0:y0 + h + 1, x0:x0 + w + 1]
    return (a[:-1, :-1] * (1 - fy) * (1 - fx) + a[:-1, 1:] * (1 - fy) * fx + a[1:, :-1] * fy * (1 - fx) +
            a[1:, 1:] * fy * fx)


def pan_path(n_frames: int, seed: int = 0, whip_at=None, whip=(0.0, 70.0)) -> np.ndarray:
    """Camera offsets [n, 2] (dy, dx): slow drift, a steady pan, optional whip pans (a jump of
    `whip` px between two frames), and a still stretch."""
    rng = np.random.default_rng(seed)
    off = np.zeros((n_frames, 2))
    pos = np.array([60.0, 60.0])
    for f in range(n_frames):
        phase = f / max(n_frames - 1, 1)
        if phase < 0.25:
            v = rng.normal(0, 0.4, 2)                     # jitter / drift
        elif phase < 0.42:
            v = np.array([1.3, 34.0]) + rng.normal(0, 0.6, 2)  # fast steady pan (> 30 px / frame)
        elif phase < 0.6:
            v = np.array([-2.0, 56.0]) + rng.normal(0, 0.6, 2)  # faster pan (> 50 px / frame: resets)
        elif phase < 0.8:
            v = np.array([0.5, 6.5]) + rng.normal(0, 0.3, 2)
        else:
            v = np.zeros(2)                               # still camera
        if whip_at is not None and f in whip_at:
            v = v + np.asarray(whip)
        pos = pos + v
        off[f] = pos
    return off


def camera_sequence(seed: int, n_frames: int, h: int = 256, w: int = 320, whip_at=(9,), n_targets: int = 4):
    """uint8 BGR frames [n, h, w, 3] of a panning camera over a world, plus the offsets."""
    rng = np.random.default_rng(seed + 1000)
    off = pan_path(n_frames, seed, whip_at=whip_at)
    span = off.max(axis=0) - off.min(axis=0)
    world = make_world(seed, int(h + span[0] + 120), int(w + span[1] + 120))
    off = off - off.min(axis=0) + 40
    tgt = rng.uniform([20, 20], [h - 20, w - 20], (n_targets, 2))
    tv = rng.normal(0, 2.5, (n_targets, 2))
    frames = np.empty((n_frames, h, w, 3), np.uint8)
    tint = rng.uniform(0.85, 1.15, 3)
    for f in range(n_frames):
        g = _sample(world, off[f, 0], off[f, 1], h, w)
        tgt += tv
        for (ty, tx) in tgt:
            y, x = int(ty) % (h - 6), int(tx) % (w - 8)
            g[y:y + 4, x:x + 7] = 235
        g = g + rng.normal(0, 1.5, g.shape)
        frames[f] = np.clip(np.stack([g * tint[0], g * tint[1], g * tint[2]], -1), 0, 255).astype(np.uint8)
    return frames, off
