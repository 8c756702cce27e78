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

    def frames_torch(self, t0: int, n: int, device, chunk: int = 32):
        """n consecutive frames rendered with torch on `device` (benchmark / large-test input
        setup; statistically the same scene as ``frame``, not bit-identical to it).

        Vectorised over frames and targets: every target's ellipse is evaluated on a fixed
        24x20 patch around its centre, and a pixel covered by several targets takes the one
        with the highest index (= the last one drawn by the per-target loop of ``frame``),
        via a scatter-max of target indices.  Deterministic on a given device."""
        import torch

        H, W, K = self.H, self.W, self.K
        gen = torch.Generator(device=device)
        gen.manual_seed(int(self.seed) * 1000003 + int(t0))
        grad = torch.linspace(60.0, 110.0, H, device=device)[:, None]
        out = torch.empty((n, H, W, 3), dtype=torch.uint8, device=device)
        PW, PH = 24, 20  # patch covers int(c - a) - 1 .. int(c + a) + 1 for a <= 10, b <= 8
        a = torch.as_tensor(self.w / 2, dtype=torch.float32, device=device)
        b = torch.as_tensor(self.h / 2, dtype=torch.float32, device=device)
        inten = torch.as_tensor(self.intensity, dtype=torch.float32, device=device)
        kidx = torch.arange(K, device=device)
        ox = torch.arange(PW, device=device)
        oy = torch.arange(PH, device=device)
        for c0 in range(0, n, chunk):
            m = min(chunk, n - c0)
            ts = np.arange(t0 + c0, t0 + c0 + m)
            g = grad + 4.0 * torch.randn((m, H, W), generator=gen, device=device)
            if K:
                pos = torch.as_tensor(self.pos[ts], dtype=torch.float32, device=device)  # [m, K, 2]
                vis = torch.as_tensor(self.visible[ts], device=device)  # [m, K]
                cx, cy = pos[..., 0], pos[..., 1]
                x0 = torch.trunc(cx - a).long() - 1
                y0 = torch.trunc(cy - b).long() - 1
                px = x0[..., None] + ox  # [m, K, PW]
                py = y0[..., None] + oy  # [m, K, PH]
                ex = ((px.float() + 0.5 - cx[..., None]) / a[:, None]) ** 2
                ey = ((py.float() + 0.5 - cy[..., None]) / b[:, None]) ** 2
                inside = (ey[..., :, None] + ex[..., None, :]) <= 1.0  # [m, K, PH, PW]
                inside &= ((px >= 0) & (px < W))[..., None, :] & ((py >= 0) & (py < H))[..., :, None]
                inside &= vis[..., None, None]
                fi = torch.arange(m, device=device)[:, None, None, None]
                lin = (fi * H + py[..., :, None]) * W + px[..., None, :]
                lab = torch.full((m * H * W,), -1, dtype=torch.long, device=device)
                lab.scatter_reduce_(0, lin[inside], kidx.view(1, K, 1, 1).expand_as(lin)[inside], reduce="amax")
                lab = lab.view(m, H, W)
                g = torch.where(lab >= 0, inten[lab.clamp(min=0)], g)
            out[c0:c0 + m] = g.round().clamp(0, 255).to(torch.uint8)[..., None].expand(m, H, W, 3)
        return out
