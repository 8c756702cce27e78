"""Synthetic infrared-like scenes for the detect-and-track path.

The reference's video and trained weights are not available, so every benchmark and
parity run uses seeded synthetic sequences:
  * 640x512 (W x H) uint8 BGR frames, three equal channels; background is a vertical
    gradient 60 -> 110 plus N(0, 4^2) noise;
  * K bright ellipses (intensity 200-255, w 6-20 px, h 4-16 px) moving with constant
    velocity (|v| <= 2 px/frame), bouncing at the borders;
  * occlusion bursts of L frames, L drawn from {1, 30, 149, 150} (150 reaches the
    deletion boundary of max_lost_frames=150);
  * ``numpy.random.default_rng(seed=stream_id)`` (seed 0 = the training run's seed,
    small_target_detection/yolov8_small_aircraft/args.yaml).
Detections for tracker-only runs ("GT-injected") are jittered float32 boxes with
conf ~ U(0.3, 0.95), dropped while a target is occluded.
"""
from __future__ import annotations

import numpy as np

OCCLUSION_LENGTHS = (1, 30, 149, 150)


class Scene:
    def __init__(self, seed: int = 0, n_targets: int = 16, n_frames: int = 650, width: int = 640,
                 height: int = 512, occlusion_lengths=OCCLUSION_LENGTHS, occlusions_per_target: float = 0.6,
                 max_speed: float = 2.0):
        rng = np.random.default_rng(seed)
        self.seed, self.K, self.T, self.W, self.H = seed, n_targets, n_frames, width, height
        K = n_targets
        self.w = rng.uniform(6, 20, K)
        self.h = rng.uniform(4, 16, K)
        self.intensity = rng.uniform(200, 255, K)
        speed = rng.uniform(0.2, max_speed, K)
        ang = rng.uniform(-np.pi, np.pi, K)
        v = np.stack([speed * np.cos(ang), speed * np.sin(ang)], 1)
        p = np.stack([rng.uniform(20, width - 20, K), rng.uniform(20, height - 20, K)], 1)
        pos = np.zeros((n_frames, K, 2))
        for t in range(n_frames):
            pos[t] = p
            p = p + v
            for ax, lim in ((0, width), (1, height)):
                lo = p[:, ax] < 10
                hi = p[:, ax] > lim - 10
                v[lo | hi, ax] *= -1
                p[:, ax] = np.clip(p[:, ax], 10, lim - 10)
        self.pos = pos
        vis = np.ones((n_frames, K), bool)
        for k in range(K):
            if rng.random() < occlusions_per_target:
                L = int(rng.choice(occlusion_lengths))
                start = int(rng.integers(5, max(6, n_frames - 5)))
                vis[start:start + L, k] = False
        self.visible = vis

    # -- ground truth ------------------------------------------------------------
    def boxes(self, t: int) -> np.ndarray:
        c = self.pos[t]
        return np.stack([c[:, 0] - self.w / 2, c[:, 1] - self.h / 2, c[:, 0] + self.w / 2, c[:, 1] + self.h / 2], 1)

    def detections(self, t: int, jitter: float = 0.5, conf_range=(0.3, 0.95)) -> list:
        """GT-injected detections of frame t as the reference driver builds them: a list of
        [x1, y1, x2, y2, conf] with np.float32 elements (aircraft_detection_tracking.py:99-106)."""
        rng = np.random.default_rng((self.seed, t, 7))
        b = self.boxes(t) + rng.normal(0, jitter, (self.K, 4))
        conf = rng.uniform(*conf_range, self.K)
        b = b.astype(np.float32)
        conf = conf.astype(np.float32)
        order = rng.permutation(self.K)
        return [[b[k, 0], b[k, 1], b[k, 2], b[k, 3], conf[k]] for k in order if self.visible[t, k]]

    def detections_array(self, t: int, **kw) -> np.ndarray:
        d = self.detections(t, **kw)
        return np.array(d, dtype=np.float32).reshape(-1, 5)

    # -- rendering ---------------------------------------------------------------
    def frame(self, t: int) -> np.ndarray:
        """uint8 BGR H x W x 3 frame (numpy; the parity/oracle input)."""
        rng = np.random.default_rng((self.seed, t, 3))
        H, W = self.H, self.W
        g = np.linspace(60.0, 110.0, H)[:, None] + rng.normal(0.0, 4.0, (H, W))
        for k in range(self.K):
            if not self.visible[t, k]:
                continue
            cx, cy = self.pos[t, k]
            a, b = self.w[k] / 2, self.h[k] / 2
            x0, x1 = max(int(cx - a) - 1, 0), min(int(cx + a) + 2, W)
            y0, y1 = max(int(cy - b) - 1, 0), min(int(cy + b) + 2, H)
            yy, xx = np.mgrid[y0:y1, x0:x1]
            m = ((xx + 0.5 - cx) / a) ** 2 + ((yy + 0.5 - cy) / b) ** 2 <= 1.0
            g[y0:y1, x0:x1][m] = self.intensity[k]
        img = np.clip(np.rint(g), 0, 255).astype(np.uint8)
        return np.repeat(img[:, :, None], 3, axis=2)

    def frames_torch(self, t0: int, n: int, device):
        """n consecutive frames rendered on the GPU with torch (benchmark input setup only;
        statistically the same scene, not bit-identical to ``frame``)."""
        import torch

        H, W = self.H, self.W
        gen = torch.Generator(device=device)
        gen.manual_seed(int(self.seed) * 1000003 + int(t0))
        yy = torch.arange(H, device=device, dtype=torch.float32)[:, None] + 0.5
        xx = torch.arange(W, device=device, dtype=torch.float32)[None, :] + 0.5
        grad = torch.linspace(60.0, 110.0, H, device=device)[:, None].expand(H, W)
        out = torch.empty((n, H, W, 3), dtype=torch.uint8, device=device)
        for i in range(n):
            t = t0 + i
            g = grad + 4.0 * torch.randn((H, W), generator=gen, device=device)
            for k in np.nonzero(self.visible[t])[0]:
                cx, cy = self.pos[t, k]
                a, b = self.w[k] / 2, self.h[k] / 2
                x0, x1 = max(int(cx - a) - 1, 0), min(int(cx + a) + 2, W)
                y0, y1 = max(int(cy - b) - 1, 0), min(int(cy + b) + 2, H)
                m = ((xx[:, x0:x1] - cx) / a) ** 2 + ((yy[y0:y1] - cy) / b) ** 2 <= 1.0
                g[y0:y1, x0:x1] = torch.where(m, torch.tensor(float(self.intensity[k]), device=device),
                                              g[y0:y1, x0:x1])
            out[i] = g.round().clamp(0, 255).to(torch.uint8)[:, :, None].expand(H, W, 3)
        return out
