"""CPU check that the arithmetic the HIP tracker kernel implements (csrc/tracker.hip) is
bit-identical to the numpy oracle (given the same arctan2; numpy and the GPU libm differ
in the last ulp there, which the GPU parity tests allow for): the per-coordinate 2x2 filter formulas, the motion
statistics (sequential axis-0 sums, numpy pairwise 1-D sums) and the mixed f32/f64 IoU.
This is a straight Python transcription of the kernel's device functions."""
import math

import numpy as np
import pytest

from oracle.tracker_ref import RefTrack, ref_iou

f32 = np.float32
QP = [0.1, 0.1, 0.01, 0.01]
QV = [0.1, 0.1, 0.001, 0.001]


class KTrack:
    def __init__(self, b):
        cx, cy = (b[0] + b[2]) / f32(2), (b[1] + b[3]) / f32(2)
        w, h = b[2] - b[0], b[3] - b[1]
        self.x = [float(cx), float(cy), float(w), float(h), 0.0, 0.0, 0.0, 0.0]
        self.P = [[50.0, 0.0, 0.0, 100.0 if c < 2 else 1.0] for c in range(4)]
        self.vh, self.ang = [], []
        self.ma = [0.0] * 8

    def predict(self):
        for c in range(4):
            self.x[c] = self.x[c] + self.x[c + 4]
            p, a, b, v = self.P[c]
            app, apv = p + b, a + v
            self.P[c] = [(app + apv) + QP[c], apv + 0.0, (b + v) + 0.0, v + QV[c]]

    def update(self, box):
        cx, cy = (box[0] + box[2]) / f32(2), (box[1] + box[3]) / f32(2)
        z = [float(cx), float(cy), float(box[2] - box[0]), float(box[3] - box[1])]
        for c in range(4):
            p, a, b, v = self.P[c]
            y = z[c] - self.x[c]
            inv = 1.0 / (p + 10.0)
            kp, kv = p * inv, b * inv
            self.x[c] = self.x[c] + kp * y
            self.x[c + 4] = self.x[c + 4] + kv * y
            ikh, nkv = 1.0 - kp, -kv
            self.P[c] = [ikh * p, ikh * a, nkv * p + b, nkv * a + v]
        self.vh = (self.vh + [(self.x[4], self.x[5])])[-50:]
        self.ang = (self.ang + [float(np.arctan2(self.x[5], self.x[4]))])[-50:]
        self.analyze()

    @staticmethod
    def pairwise(a):
        n = len(a)
        if n < 8:
            r = 0.0
            for v in a:
                r += v
            return r
        r = list(a[:8])
        i = 8
        while i < n - n % 8:
            for j in range(8):
                r[j] += a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i]
            i += 1
        return res

    def analyze(self):
        n = len(self.vh)
        if n < 5:
            return
        mean, sd = [], []
        for j in range(2):
            acc = self.vh[0][j]
            for k in range(1, n):
                acc += self.vh[k][j]
            mean.append(acc / n)
        for j in range(2):
            d = self.vh[0][j] - mean[j]
            acc = d * d
            for k in range(1, n):
                d = self.vh[k][j] - mean[j]
                acc += d * d
            sd.append(math.sqrt(acc / n))
        speed = math.sqrt(mean[0] * mean[0] + mean[1] * mean[1])
        direction = float(np.arctan2(mean[1], mean[0]))
        ss = 1.0 / (1.0 + ((0.0 + sd[0]) + sd[1]) / 2.0)
        dch = []
        for k in range(n - 1):
            c = self.ang[k + 1] - self.ang[k]
            if not abs(c) < math.pi:
                c = c - 2.0 * math.pi * (1.0 if c > 0 else -1.0)
            dch.append(c)
        m = n - 1
        dm = self.pairwise(dch) / m
        dstd = math.sqrt(self.pairwise([(d - dm) * (d - dm) for d in dch]) / m)
        stab = (ss + 1.0 / (1.0 + dstd * 10.0)) / 2.0
        self.ma = [mean[0], mean[1], sd[0], sd[1], direction, speed, stab, stab * min(n / 30.0, 1.0)]


@pytest.mark.parametrize("seed", range(6))
def test_kernel_filter_formulas_bitwise(seed):
    rng = np.random.default_rng(seed)
    b0 = [f32(v) for v in (100 + rng.normal(), 100 + rng.normal(), 110 + rng.normal(), 108 + rng.normal())]
    r, k = RefTrack(b0, "T", 150), KTrack(b0)
    vx, vy = rng.uniform(-2, 2, 2)
    for t in range(120):
        r.predict()
        k.predict()
        if rng.random() < 0.75:
            cx, cy = 105 + vx * t + rng.normal(0, 0.7), 104 + vy * t + rng.normal(0, 0.7)
            box = [f32(cx - 5 + rng.normal(0, .3)), f32(cy - 4), f32(cx + 5), f32(cy + 4 + rng.normal(0, .3))]
            r.update(box)
            k.update(box)
        assert r.x.tolist() == k.x, t
        for c in range(4):
            assert [r.P[c, c], r.P[c, c + 4], r.P[c + 4, c], r.P[c + 4, c + 4]] == k.P[c], (t, c)
        ma = r.motion_analysis
        ref_ma = [*ma["velocity_avg"], *ma["velocity_std"], ma["direction"], ma["speed"], ma["stability_score"],
                  ma["prediction_confidence"]]
        assert [float(v) for v in ref_ma] == k.ma, t


def _kernel_iou(d, t):
    """Transcription of iou_mixed<float> in tracker.hip."""
    tx1, ty1 = t[0] > float(d[0]), t[1] > float(d[1])
    tx2, ty2 = t[2] < float(d[2]), t[3] < float(d[3])
    ix1 = t[0] if tx1 else float(d[0])
    iy1 = t[1] if ty1 else float(d[1])
    ix2 = t[2] if tx2 else float(d[2])
    iy2 = t[3] if ty2 else float(d[3])
    if ix2 <= ix1 or iy2 <= iy1:
        return 0.0
    wdt, hdt = not tx1 and not tx2, not ty1 and not ty2
    w = float(f32(d[2] - d[0])) if wdt else ix2 - ix1
    h = float(f32(d[3] - d[1])) if hdt else iy2 - iy1
    inter = float(f32(w) * f32(h)) if (wdt and hdt) else w * h
    a1 = (d[2] - d[0]) * (d[3] - d[1])
    a2 = (t[2] - t[0]) * (t[3] - t[1])
    u = (float(a1) + a2) - inter
    if u <= 0.0:
        return 0.0
    return inter / u


def test_kernel_mixed_iou_bitwise():
    rng = np.random.default_rng(0)
    n = 0
    for _ in range(20000):
        c = rng.uniform(0, 600, 2)
        d = [f32(v) for v in (c[0], c[1], c[0] + rng.uniform(1, 30), c[1] + rng.uniform(1, 30))]
        o = rng.normal(0, 6, 2)
        wh = rng.uniform(1, 30, 2)
        if rng.random() < 0.2:  # exact coordinate ties with the detection
            t = np.array([float(d[0]), float(d[1]), float(d[0]) + wh[0], float(d[1]) + wh[1]])
        else:
            t = np.array([c[0] + o[0], c[1] + o[1], c[0] + o[0] + wh[0], c[1] + o[1] + wh[1]])
        a, b = ref_iou(d, t), _kernel_iou(d, t)
        assert a == b
        n += a > 0
    assert n > 1000
