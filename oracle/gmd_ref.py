"""TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline) -- never the product path.

numpy restatement of the global camera-motion detector,
camera_motion_compensation/global_motion_detector.py:11-288 (GlobalMotionDetector, method
'optical_flow', the default and the one MotionCompensatedMultiTracker uses,
motion_compensated_multi_tracker.py:31,44), including the OpenCV calls it makes:

  cv2.cvtColor(frame, COLOR_BGR2GRAY)              (:79, :82)
  cv2.goodFeaturesToTrack(prev_gray, maxCorners=200, qualityLevel=0.01, minDistance=15,
                          blockSize=7)              (:49-55, :116)
  cv2.calcOpticalFlowPyrLK(prev_gray, curr_gray, corners, None, winSize=(21, 21), maxLevel=3,
                           criteria=(EPS|COUNT, 30, 0.01))   (:43-47, :122-124)

cv2 is not installed in this image and the reference may not be run here, so the
OpenCV part is restated from OpenCV 4.x's published algorithms (imgproc color.cpp RGB2Gray,
corner.cpp cornerMinEigenVal, featureselect.cpp goodFeaturesToTrack, pyramids.cpp pyrDown,
video lkpyramid.cpp buildOpticalFlowPyramid / calcSharrDeriv / LKTrackerInvoker) and is
PARITY UNPINNED against cv2 itself.  Where OpenCV's result depends on its SIMD float
accumulation order, this restatement fixes an exact order instead (documented per function);
the device kernels (csrc/gmd.hip) reproduce this restatement bit for bit.  The numpy
post-processing of the reference (median / percentile / mean / norm / arctan2 on float32, NEP 50
scalar rules) is restated with numpy itself.
"""
from __future__ import annotations

from collections import deque

import numpy as np

WIN = 21            # lk_params winSize (:44)
MAX_LEVEL = 3       # lk_params maxLevel (:45)
MAX_COUNT = 30      # criteria count (:46)
EPSILON = 0.01      # criteria eps (:46)
MIN_EIG_THR = np.float32(1e-4)  # calcOpticalFlowPyrLK default minEigThreshold
MAX_CORNERS, QUALITY, MIN_DIST, BLOCK = 200, 0.01, 15.0, 7  # feature_params (:50-55)
FLT_EPS = np.float32(1.1920928955078125e-07)
_F = np.float32


def _refl(i, n):
    """BORDER_REFLECT_101 index (gfedcb|abcdefgh|gfedcba) for |overflow| < n."""
    i = np.where(i < 0, -i, i)
    return np.where(i >= n, 2 * n - 2 - i, i)


# ------------------------------------------------------------------ cvtColor BGR2GRAY
def bgr_to_gray(frame: np.ndarray) -> np.ndarray:
    """color.cpp RGB2Gray<uchar>: fixed point, yuv_shift 14, coefficients R 4899 G 9617 B 1868."""
    f = frame.astype(np.int32)
    return ((f[..., 0] * 1868 + f[..., 1] * 9617 + f[..., 2] * 4899 + (1 << 13)) >> 14).astype(np.uint8)


# ------------------------------------------------------------------ goodFeaturesToTrack
def min_eig(gray: np.ndarray, block: int = BLOCK) -> np.ndarray:
    """cornerMinEigenVal(gray, blockSize=7, ksize=3) (corner.cpp cornerEigenValsVecs, MINEIGENVAL).

    OpenCV: Sobel(ksize 3, BORDER_REFLECT_101) with scale 1/(4*7*255) in float, products, an
    unnormalised 7x7 boxFilter (BORDER_REFLECT_101) of the products, then per pixel
    a = cxx/2, b = cxy, c = cyy/2, (a + c) - sqrt((a - c)^2 + b^2) in float.  Restated with the
    Sobel responses and the box sums in exact integers and one rounding per covariance entry:
    c.. = float32(S.. * scale^2) (the cv2 value differs at the ulp level by its float sums)."""
    h, w = gray.shape
    g = gray.astype(np.int64)
    ys, xs = np.arange(h), np.arange(w)
    gp = g[_refl(ys - 1, h)][:, :], g, g[_refl(ys + 1, h)]
    xm, xp = _refl(xs - 1, w), _refl(xs + 1, w)
    ix = (gp[0][:, xp] - gp[0][:, xm]) + 2 * (gp[1][:, xp] - gp[1][:, xm]) + (gp[2][:, xp] - gp[2][:, xm])
    iy = (gp[2][:, xm] + 2 * gp[2] + gp[2][:, xp]) - (gp[0][:, xm] + 2 * gp[0] + gp[0][:, xp])
    r = block // 2

    def box(a):
        out = np.zeros_like(a)
        for dy in range(-r, r + 1):
            rows = a[_refl(ys + dy, h)]
            for dx in range(-r, r + 1):
                out += rows[:, _refl(xs + dx, w)]
        return out

    s2 = 1.0 / (4.0 * block * 255.0) ** 2
    cxx = (box(ix * ix) * s2).astype(np.float32)
    cxy = (box(ix * iy) * s2).astype(np.float32)
    cyy = (box(iy * iy) * s2).astype(np.float32)
    a = cxx * _F(0.5)
    c = cyy * _F(0.5)
    d = a - c
    return ((a + c) - np.sqrt(d * d + cxy * cxy)).astype(np.float32)


def good_features(gray: np.ndarray, max_corners=MAX_CORNERS, quality=QUALITY, min_distance=MIN_DIST,
                  block=BLOCK, return_info=False):
    """goodFeaturesToTrack (featureselect.cpp): threshold TOZERO at maxVal * qualityLevel, 3x3
    dilate (constant border = ignored), local maxima of the interior (1 <= x <= w-2,
    1 <= y <= h-2), std::sort by (value desc, address desc) (greaterThanPtr), then the greedy
    minDistance pass over a grid of cell_size = cvRound(minDistance) cells (checks the 3x3
    neighbouring cells, dx*dx + dy*dy < minDistance^2) until maxCorners are kept.
    Returns float32 [N, 1, 2] (x, y) or None when no corner is found (cv2's empty output)."""
    h, w = gray.shape
    eig = min_eig(gray, block)
    max_val = float(eig.max())
    thr = np.float32(max_val * quality)
    t = np.where(eig > thr, eig, _F(0))
    pad = np.full((h + 2, w + 2), -np.inf, np.float32)
    pad[1:-1, 1:-1] = t
    dil = np.max(np.stack([pad[dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)]), axis=0)
    inner = np.zeros((h, w), bool)
    inner[1:h - 1, 1:w - 1] = True
    cand = inner & (t != 0) & (t == dil)
    yy, xx = np.nonzero(cand)
    val = t[yy, xx]
    addr = yy.astype(np.int64) * w + xx
    order = np.lexsort((-addr, -val.astype(np.float64)))
    yy, xx = yy[order], xx[order]
    cell = int(np.round(min_distance))
    gw, gh = (w + cell - 1) // cell, (h + cell - 1) // cell
    grid = [[] for _ in range(gw * gh)]
    md2 = min_distance * min_distance
    out = []
    for y, x in zip(yy.tolist(), xx.tolist()):
        xc, yc = x // cell, y // cell
        good = True
        for gy in range(max(0, yc - 1), min(gh - 1, yc + 1) + 1):
            for gx in range(max(0, xc - 1), min(gw - 1, xc + 1) + 1):
                for (px, py) in grid[gy * gw + gx]:
                    dx, dy = np.float32(x - px), np.float32(y - py)
                    if float(dx * dx + dy * dy) < md2:
                        good = False
                        break
                if not good:
                    break
            if not good:
                break
        if good:
            grid[yc * gw + xc].append((x, y))
            out.append((x, y))
            if len(out) == max_corners:
                break
    corners = np.asarray(out, np.float32).reshape(-1, 1, 2) if out else None
    if return_info:
        return corners, {"max_val": max_val, "n_candidates": int(len(yy)), "eig": eig}
    return corners


# ------------------------------------------------------------------ calcOpticalFlowPyrLK
def pyr_down(img: np.ndarray) -> np.ndarray:
    """pyrDown (pyramids.cpp) for uchar: 5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101, integer
    sums with one (+128) >> 8 rounding; dst size ((w+1)/2, (h+1)/2)."""
    h, w = img.shape
    dh, dw = (h + 1) // 2, (w + 1) // 2
    k = (1, 4, 6, 4, 1)
    src = img.astype(np.int64)
    xs = 2 * np.arange(dw)
    rows = np.zeros((h, dw), np.int64)
    for j in range(5):
        rows += k[j] * src[:, _refl(xs + j - 2, w)]
    ys = 2 * np.arange(dh)
    acc = np.zeros((dh, dw), np.int64)
    for i in range(5):
        acc += k[i] * rows[_refl(ys + i - 2, h)]
    return ((acc + 128) >> 8).astype(np.uint8)


def pyramid_levels(h: int, w: int, win: int = WIN, max_level: int = MAX_LEVEL) -> int:
    """buildOpticalFlowPyramid's level count: stop once the next level would be <= winSize."""
    level = 0
    while level < max_level:
        w2, h2 = (w + 1) // 2, (h + 1) // 2
        if w2 <= win or h2 <= win:
            break
        w, h, level = w2, h2, level + 1
    return level


def build_pyramid(gray: np.ndarray, levels: int) -> list:
    pyr = [gray]
    for _ in range(levels):
        pyr.append(pyr_down(pyr[-1]))
    return pyr


def scharr_deriv(img: np.ndarray):
    """calcSharrDeriv (lkpyramid.cpp): vertical [3 10 3] / [-1 0 1] pass, then horizontal
    [-1 0 1] / [3 10 3], BORDER_REFLECT_101, int16 results (|d| <= 4080)."""
    h, w = img.shape
    s = img.astype(np.int64)
    ys, xs = np.arange(h), np.arange(w)
    r0, r2 = s[_refl(ys - 1, h)], s[_refl(ys + 1, h)]
    t0 = (r0 + r2) * 3 + s * 10
    t1 = r2 - r0
    xm, xp = _refl(xs - 1, w), _refl(xs + 1, w)
    dx = t0[:, xp] - t0[:, xm]
    dy = (t1[:, xp] + t1[:, xm]) * 3 + t1 * 10
    return dx, dy


def _bilinear_weights(frac_x, frac_y):
    """cvRound((1-a)(1-b) 2^14) etc. in float32, round half to even (cvRound = lrint)."""
    one = _F(1)
    scale = _F(1 << 14)
    w00 = np.rint(((one - frac_x) * (one - frac_y)) * scale).astype(np.int64)
    w01 = np.rint((frac_x * (one - frac_y)) * scale).astype(np.int64)
    w10 = np.rint(((one - frac_x) * frac_y) * scale).astype(np.int64)
    w11 = (1 << 14) - w00 - w01 - w10
    return w00, w01, w10, w11


def _gather(padded, pad, y0, x0):
    """[P, WIN+1, WIN+1] block of `padded` whose top-left is image (y0, x0)."""
    oy = np.arange(WIN + 1)
    ry = (y0[:, None] + pad + oy[None, :])
    rx = (x0[:, None] + pad + oy[None, :])
    return padded[ry[:, :, None], rx[:, None, :]]


def _interp(block, w, shift):
    w00, w01, w10, w11 = (v[:, None, None] for v in w)
    acc = (block[:, :-1, :-1] * w00 + block[:, :-1, 1:] * w01 + block[:, 1:, :-1] * w10 + block[:, 1:, 1:] * w11)
    return (acc + (1 << (shift - 1))) >> shift


def lk_track(prev_pyr, next_pyr, pts: np.ndarray, win=WIN, max_count=MAX_COUNT, eps=EPSILON):
    """LKTrackerInvoker over every level (lkpyramid.cpp), vectorised over points.

    Integer parts are exact (bilinear weights W_BITS 14, I patch descaled by 9 bits, derivatives
    by 14); the window sums A11 / A12 / A22 / b1 / b2 are accumulated exactly in int64 and
    rounded once to float32 (OpenCV accumulates in float, order set by its SIMD lanes).  Float
    steps follow the C++ expressions: minEig = (A22 + A11 - sqrt((A11-A22)^2 + 4 A12 A12)) /
    (2 * 21 * 21), delta = ((A12 b2 - A22 b1) D, (A12 b1 - A11 b2) D), convergence
    delta.ddot(delta) <= eps^2 in double, oscillation |delta + prevDelta| < 0.01 -> step back by
    half a delta.  Returns next points float32 [N, 2] and status uint8 [N]."""
    assert win == WIN
    levels = len(prev_pyr) - 1
    n = len(pts)
    pts = pts.reshape(n, 2).astype(np.float32)
    status = np.ones(n, np.uint8)
    nxt = pts.copy()
    half = _F((win - 1) * 0.5)
    pad = WIN + 2
    for level in range(levels, -1, -1):
        I, J = prev_pyr[level], next_pyr[level]
        rows, cols = I.shape
        dxI, dyI = scharr_deriv(I)
        Ip = np.pad(I.astype(np.int64), pad, mode="reflect")
        Jp = np.pad(J.astype(np.int64), pad, mode="reflect")
        DXp = np.pad(dxI, pad)
        DYp = np.pad(dyI, pad)
        prev = pts * _F(1.0 / (1 << level))
        cur = prev.copy() if level == levels else nxt * _F(2)
        nxt = cur.copy()
        p = prev - half
        ip = np.floor(p).astype(np.int64)
        oob = (ip[:, 0] < -win) | (ip[:, 0] >= cols) | (ip[:, 1] < -win) | (ip[:, 1] >= rows)
        if level == 0:
            status[oob] = 0
        act = ~oob
        if not act.any():
            continue
        idx = np.nonzero(act)[0]
        a = (p[idx, 0] - ip[idx, 0].astype(np.float32)).astype(np.float32)
        b = (p[idx, 1] - ip[idx, 1].astype(np.float32)).astype(np.float32)
        wts = _bilinear_weights(a, b)
        y0, x0 = ip[idx, 1], ip[idx, 0]
        ival = _interp(_gather(Ip, pad, y0, x0), wts, 9)
        ixv = _interp(_gather(DXp, pad, y0, x0), wts, 14)
        iyv = _interp(_gather(DYp, pad, y0, x0), wts, 14)
        fs = _F(1.0 / (1 << 20))
        A11 = (ixv * ixv).sum(axis=(1, 2)).astype(np.float32) * fs
        A12 = (ixv * iyv).sum(axis=(1, 2)).astype(np.float32) * fs
        A22 = (iyv * iyv).sum(axis=(1, 2)).astype(np.float32) * fs
        D = A11 * A22 - A12 * A12
        dd = A11 - A22
        min_eig = ((A22 + A11) - np.sqrt(dd * dd + (_F(4) * A12) * A12)) / _F(2 * win * win)
        bad = (min_eig < MIN_EIG_THR) | (D < FLT_EPS)
        if level == 0:
            status[idx[bad]] = 0
        keep = ~bad
        idx, ival, ixv, iyv = idx[keep], ival[keep], ixv[keep], iyv[keep]
        A11, A12, A22, D = A11[keep], A12[keep], A22[keep], D[keep]
        D = _F(1) / D
        npt = cur[idx] - half
        pdelta = np.zeros((len(idx), 2), np.float32)
        live = np.ones(len(idx), bool)
        eps2 = eps * eps
        for j in range(max_count):
            if not live.any():
                break
            li = np.nonzero(live)[0]
            inx = np.floor(npt[li]).astype(np.int64)
            oob = (inx[:, 0] < -win) | (inx[:, 0] >= cols) | (inx[:, 1] < -win) | (inx[:, 1] >= rows)
            if level == 0:
                status[idx[li[oob]]] = 0
            live[li[oob]] = False
            li, inx = li[~oob], inx[~oob]
            if len(li) == 0:
                break
            a = (npt[li, 0] - inx[:, 0].astype(np.float32)).astype(np.float32)
            b = (npt[li, 1] - inx[:, 1].astype(np.float32)).astype(np.float32)
            wts = _bilinear_weights(a, b)
            jval = _interp(_gather(Jp, pad, inx[:, 1], inx[:, 0]), wts, 9)
            diff = jval - ival[li]
            b1 = (diff * ixv[li]).sum(axis=(1, 2)).astype(np.float32) * fs
            b2 = (diff * iyv[li]).sum(axis=(1, 2)).astype(np.float32) * fs
            dxs = (A12[li] * b2 - A22[li] * b1) * D[li]
            dys = (A12[li] * b1 - A11[li] * b2) * D[li]
            npt[li, 0] += dxs
            npt[li, 1] += dys
            nxt[idx[li], 0] = npt[li, 0] + half
            nxt[idx[li], 1] = npt[li, 1] + half
            conv = (dxs.astype(np.float64) * dxs + dys.astype(np.float64) * dys) <= eps2
            osc = np.zeros(len(li), bool)
            if j > 0:
                osc = (np.abs((dxs + pdelta[li, 0]).astype(np.float64)) < 0.01) & \
                      (np.abs((dys + pdelta[li, 1]).astype(np.float64)) < 0.01) & ~conv
                oi = idx[li[osc]]
                nxt[oi, 0] -= dxs[osc] * _F(0.5)
                nxt[oi, 1] -= dys[osc] * _F(0.5)
            pdelta[li, 0], pdelta[li, 1] = dxs, dys
            live[li[conv | osc]] = False
    return nxt, status


def optical_flow(prev_gray, curr_gray, corners):
    levels = min(pyramid_levels(*prev_gray.shape), pyramid_levels(*curr_gray.shape))
    return lk_track(build_pyramid(prev_gray, levels), build_pyramid(curr_gray, levels), corners.reshape(-1, 2))


# ------------------------------------------------------------------ GlobalMotionDetector
class RefGlobalMotionDetector:
    """GlobalMotionDetector(method='optical_flow') (global_motion_detector.py:11-288)."""

    def __init__(self, method="optical_flow"):
        if method != "optical_flow":
            raise NotImplementedError("feature_matching / hybrid need cv2 ORB + RANSAC findHomography")
        self.method = method
        self.prev_gray = None
        self.motion_history = deque(maxlen=10)
        self.motion_vectors = deque(maxlen=5)
        self.global_motion_threshold = 30.0
        self.reset_motion_threshold = 50.0
        self.consistency_threshold = 0.7
        self.reset_stats()
        self.last_debug = {}

    def reset_stats(self):
        self.stats = {"total_detections": 0, "motion_events": 0, "reset_triggers": 0, "avg_motion_magnitude": 0.0}

    def detect_motion(self, frame):
        """:67-111"""
        if self.prev_gray is None:
            self.prev_gray = bgr_to_gray(frame)
            return False, 0.0, np.array([0.0, 0.0]), False
        curr_gray = bgr_to_gray(frame)
        result = self._detect_by_optical_flow(curr_gray)
        self.prev_gray = curr_gray
        self.stats["total_detections"] += 1
        is_motion, mag, vec, should_reset = result
        if is_motion:
            self.stats["motion_events"] += 1
        if should_reset:
            self.stats["reset_triggers"] += 1
        n = self.stats["total_detections"]
        self.stats["avg_motion_magnitude"] = (self.stats["avg_motion_magnitude"] * (n - 1) + mag) / n
        return result

    def _detect_by_optical_flow(self, curr_gray):
        """:113-169"""
        none = (False, 0.0, np.array([0.0, 0.0]), False)
        corners = good_features(self.prev_gray)
        self.last_debug = {"corners": corners, "next": None, "status": None}
        if corners is None or len(corners) < 20:
            return none
        nxt, status = optical_flow(self.prev_gray, curr_gray, corners)
        self.last_debug.update(next=nxt, status=status)
        good = status.flatten() == 1
        if np.sum(good) < 10:
            return none
        prev_points = corners[good].reshape(-1, 2)
        next_points = nxt[good].reshape(-1, 2)
        motion_vectors = next_points - prev_points
        if len(motion_vectors) > 8:
            median_motion = np.median(motion_vectors, axis=0)
            distances = np.linalg.norm(motion_vectors - median_motion, axis=1)
            inliers = distances < np.percentile(distances, 75)
            if np.sum(inliers) > 5:
                gmv = np.mean(motion_vectors[inliers], axis=0)
                mag = np.linalg.norm(gmv)
                self.motion_history.append(mag)
                self.motion_vectors.append(gmv)
                is_motion = mag > self.global_motion_threshold
                should_reset = mag > self.reset_motion_threshold
                if len(self.motion_vectors) >= 3:
                    consistency = self._calculate_motion_consistency(list(self.motion_vectors)[-3:])
                    self.last_debug["consistency"] = consistency
                    if consistency > self.consistency_threshold and is_motion:
                        should_reset = should_reset or mag > self.global_motion_threshold * 1.5
                return is_motion, mag, gmv, should_reset
        return none

    @staticmethod
    def _calculate_motion_consistency(vectors):
        """:241-261"""
        if len(vectors) < 2:
            return 0.0
        angles = [np.arctan2(v[1], v[0]) for v in vectors]
        diffs = []
        for i in range(1, len(angles)):
            diff = abs(angles[i] - angles[i - 1])
            if diff > np.pi:
                diff = 2 * np.pi - diff
            diffs.append(diff)
        return max(0.0, 1.0 - np.mean(diffs) / np.pi)

    def get_stats(self):
        """:263-278"""
        s = self.stats
        if s["total_detections"] > 0:
            mr = s["motion_events"] / s["total_detections"]
            rr = s["reset_triggers"] / s["total_detections"]
        else:
            mr = rr = 0.0
        return {"total_detections": s["total_detections"], "motion_events": s["motion_events"],
                "reset_triggers": s["reset_triggers"], "motion_detection_rate": f"{mr:.1%}",
                "reset_trigger_rate": f"{rr:.1%}", "avg_motion_magnitude": f"{s['avg_motion_magnitude']:.2f}px"}
