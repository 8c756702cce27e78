"""TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline) -- never the product path.

numpy restatement of BoT-SORT's default global motion compensation,
ultralytics/trackers/utils/gmc.py:278-345 (GMC(method='sparseOptFlow', downscale=2), the
cfg/trackers/botsort.yaml:17 default), including the OpenCV calls it makes:

  cv2.cvtColor(raw, COLOR_BGR2GRAY)                                          (:296)
  cv2.resize(frame, (w // 2, h // 2))  (INTER_LINEAR at an exact 1/2 scale: resize.cpp switches
                                        to INTER_AREA's integer fast path, (a+b+c+d+2) >> 2)  (:301)
  cv2.goodFeaturesToTrack(frame, maxCorners=1000, qualityLevel=0.01, minDistance=1, blockSize=3,
                          useHarrisDetector=False)                          (:78-80, :304)
  cv2.calcOpticalFlowPyrLK(prevFrame, frame, prevKeyPoints, None)  (defaults: winSize 21x21,
                          maxLevel 3, criteria (COUNT|EPS, 30, 0.01))       (:314)
  cv2.estimateAffinePartial2D(prevPoints, currPoints, cv2.RANSAC)  (defaults: reprojection
                          threshold 3, maxIters 2000, confidence 0.99, refineIters 10) (:329)

The corner and Lucas-Kanade stages are oracle/gmd_ref.py's restatements with these parameters.
estimateAffinePartial2D is restated from OpenCV 4.x calib3d ptsetreg.cpp: RANSACPointSetRegistrator
(cv::RNG seeded with (uint64)-1, 2-point subsets by rng.uniform, AffinePartial2DEstimatorCallback's
closed-form kernel and float32 reprojection error, RANSACUpdateNumIters), compressElems, then the
Levenberg-Marquardt refinement of (a, b, tx, ty) over the inliers (LMSolverImpl, 10 iterations,
eps FLT_EPSILON).  Where OpenCV's floating-point order is its own (the normal equations' sums,
the 4x4 solve by Jacobi eigen-decomposition DECOMP_EIG), this restatement fixes an order: sums over
points in the device's 256-lane order (lane t adds points t, t + 256, ... sequentially, then a
fixed pairwise tree over the lanes) and a Cholesky solve -- the same solution to rounding.  cv2 is
absent here, so parity with cv2 is UNPINNED; the device kernel (csrc/gmd.hip) reproduces this
restatement.
"""
from __future__ import annotations

import copy
import math

import numpy as np

from . import gmd_ref as G

MAX_CORNERS, QUALITY, MIN_DIST, BLOCK = 1000, 0.01, 1.0, 3  # gmc.py:78-80
RANSAC_THR, MAX_ITERS, CONFIDENCE, REFINE_ITERS = 3.0, 2000, 0.99, 10  # estimateAffinePartial2D defaults
RNG_COEFF = 4164903690
LANES = 256
FLT_EPSILON = 1.1920928955078125e-07
DBL_EPSILON = 2.220446049250313e-16
DBL_MIN = 2.2250738585072014e-308
_F = np.float32


def area_down2(gray: np.ndarray) -> np.ndarray:
    """cv2.resize(gray, (w // 2, h // 2)), INTER_LINEAR at scale exactly 1/2 (resize.cpp maps it
    to INTER_AREA's fast path): each output pixel (a + b + c + d + 2) >> 2 of its 2x2 block."""
    h, w = gray.shape
    g = gray[: 2 * (h // 2), : 2 * (w // 2)].astype(np.int32)
    s = g[0::2, 0::2] + g[0::2, 1::2] + g[1::2, 0::2] + g[1::2, 1::2]
    return ((s + 2) >> 2).astype(np.uint8)


# ------------------------------------------------------------------ ordered sums (device order)
def lane_sum(v: np.ndarray) -> float:
    """Sum of a float64 vector in the device's order: lane t accumulates v[t], v[t + 256], ...
    left to right, then the 256 lane partials are summed pairwise (o = 128, 64, ..., 1:
    p[t] += p[t + o])."""
    v = np.asarray(v, np.float64)
    n = len(v)
    p = np.zeros(LANES, np.float64)
    for k in range(0, n, LANES):
        c = v[k:k + LANES]
        p[: len(c)] = p[: len(c)] + c
    o = LANES // 2
    while o >= 1:
        p[:o] = p[:o] + p[o:2 * o]
        o //= 2
    return float(p[0])


# ------------------------------------------------------------------ cv::RNG
class CvRng:
    """cv::RNG (core/include/opencv2/core/operations.hpp): multiply-with-carry,
    next(): state = (uint64)(unsigned)state * CV_RNG_COEFF + (unsigned)(state >> 32)."""

    def __init__(self, state: int = (1 << 64) - 1):
        self.state = state & ((1 << 64) - 1)

    def next(self) -> int:
        self.state = ((self.state & 0xFFFFFFFF) * RNG_COEFF + (self.state >> 32)) & ((1 << 64) - 1)
        return self.state & 0xFFFFFFFF

    def uniform(self, a: int, b: int) -> int:
        return a if a == b else a + self.next() % (b - a)


# ------------------------------------------------------------------ RANSAC (ptsetreg.cpp)
def _kernel(f, t):
    """AffinePartial2DEstimatorCallback::runKernel: the similarity through two point pairs."""
    x1, y1, x2, y2 = (float(f[0, 0]), float(f[0, 1]), float(f[1, 0]), float(f[1, 1]))
    X1, Y1, X2, Y2 = (float(t[0, 0]), float(t[0, 1]), float(t[1, 0]), float(t[1, 1]))
    den = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2)
    d = 1.0 / den if den != 0.0 else math.copysign(math.inf, den)
    S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2))
    S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2))
    S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2))
    S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2))
    return np.array([[S0, -S1, S2], [S1, S0, S3]], np.float64)


def _errors(frm, to, M) -> np.ndarray:
    """Affine2DEstimatorCallback::computeError: the model cast to float32, squared float32 error."""
    F = M.astype(np.float32).reshape(6)
    with np.errstate(all="ignore"):
        a = F[0] * frm[:, 0] + F[1] * frm[:, 1] + F[2] - to[:, 0]
        b = F[3] * frm[:, 0] + F[4] * frm[:, 1] + F[5] - to[:, 1]
        return (a * a + b * b).astype(np.float32)


def update_num_iters(p, ep, model_points, max_iters) -> int:
    """RANSACUpdateNumIters."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, DBL_MIN)
    denom = 1.0 - math.pow(1.0 - ep, model_points)
    if denom < DBL_MIN:
        return 0
    num = math.log(num)
    denom = math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    q = num / denom
    return int(np.rint(q))  # cvRound: round half to even


def ransac_partial_affine(frm, to, thr=RANSAC_THR, max_iters=MAX_ITERS, conf=CONFIDENCE):
    """RANSACPointSetRegistrator::run with the partial-affine callback (modelPoints 2).  Returns
    (model 2x3 float64 or None, inlier mask uint8, iterations run)."""
    n = len(frm)
    if n < 2:
        return None, np.zeros(n, np.uint8), 0
    t = _F(thr * thr)
    rng = CvRng()
    niters, best, best_mask, max_good, it = max(max_iters, 1), None, np.zeros(n, np.uint8), 0, 0
    if n == 2:
        return _kernel(frm, to), np.ones(n, np.uint8), 0
    while it < niters:
        i0 = rng.uniform(0, n)  # getSubset: distinct indices (the 2-point collinearity check is vacuous)
        i1 = rng.uniform(0, n)
        while i1 == i0:
            i1 = rng.uniform(0, n)
        idx = [i0, i1]
        M = _kernel(frm[idx], to[idx])
        err = _errors(frm, to, M)
        mask = (err <= t).astype(np.uint8)
        good = int(mask.sum())
        if good > max(max_good, 1):
            best, best_mask, max_good = M, mask, good
            niters = update_num_iters(conf, (n - good) / n, 2, niters)
        it += 1
    if max_good <= 0:
        return None, np.zeros(n, np.uint8), it
    return best, best_mask, it


# ------------------------------------------------------------------ Levenberg-Marquardt
def _residuals(h, src, dst):
    """AffinePartial2DRefineCallback::compute's error vector (x residuals, y residuals)."""
    Mx, My = src[:, 0].astype(np.float64), src[:, 1].astype(np.float64)
    xi = (h[0] * Mx - h[1] * My) + h[2]
    yi = (h[1] * Mx + h[0] * My) + h[3]
    return xi - dst[:, 0].astype(np.float64), yi - dst[:, 1].astype(np.float64)


def _normal(h, src, dst):
    """J^T J and J^T r of the partial-affine residuals (J rows {x, -y, 1, 0}, {y, x, 0, 1}),
    every sum in the device order (lane_sum); also S = |r|^2."""
    Mx, My = src[:, 0].astype(np.float64), src[:, 1].astype(np.float64)
    rx, ry = _residuals(h, src, dst)
    n = float(len(src))
    sxx = lane_sum(Mx * Mx + My * My)
    sx, sy = lane_sum(Mx), lane_sum(My)
    A = np.array([[sxx, 0.0, sx, sy], [0.0, sxx, -sy, sx], [sx, -sy, n, 0.0], [sy, sx, 0.0, n]])
    v = np.array([lane_sum(Mx * rx + My * ry), lane_sum(-My * rx + Mx * ry), lane_sum(rx), lane_sum(ry)])
    S = lane_sum(rx * rx + ry * ry)
    rinf = float(max(np.max(np.abs(rx)), np.max(np.abs(ry)))) if len(src) else 0.0
    return A, v, S, rinf


def chol_solve4(A, b):
    """Cholesky solve of the 4x4 SPD system in a fixed order (device: gmd.hip chol_solve4)."""
    L = np.zeros((4, 4))
    for j in range(4):
        s = A[j, j]
        for k in range(j):
            s = s - L[j, k] * L[j, k]
        L[j, j] = math.sqrt(s) if s > 0 else math.nan
        for i in range(j + 1, 4):
            s = A[i, j]
            for k in range(j):
                s = s - L[i, k] * L[j, k]
            L[i, j] = s / L[j, j]
    y = np.zeros(4)
    for i in range(4):
        s = b[i]
        for k in range(i):
            s = s - L[i, k] * y[k]
        y[i] = s / L[i, i]
    x = np.zeros(4)
    for i in range(3, -1, -1):
        s = y[i]
        for k in range(i + 1, 4):
            s = s - L[k, i] * x[k]
        x[i] = s / L[i, i]
    return x


def _inv_diag_max(A):
    """max_i |inv(A)[i][i]| (LMSolverImpl's invert(A, DECOMP_EIG) when lambda hits 0), by the
    same Cholesky solves against the unit vectors."""
    m = DBL_EPSILON
    for i in range(4):
        e = np.zeros(4)
        e[i] = 1.0
        m = max(m, abs(chol_solve4(A, e)[i]))
    return m


def lm_refine(h, src, dst, max_iters=REFINE_ITERS, eps=FLT_EPSILON):
    """LMSolverImpl::run (calib3d levmarq.cpp, OpenCV 4.x) on Hvec = (a, b, tx, ty)."""
    x = np.asarray(h, np.float64).copy()
    A, v, S, rinf = _normal(x, src, dst)
    D = np.diag(A).copy()
    Rlo, Rhi = 0.25, 0.75
    lam, lc, it = 1.0, 0.75, 0
    while True:
        Ap = A.copy()
        for i in range(4):
            Ap[i, i] = Ap[i, i] + lam * D[i]
        d = chol_solve4(Ap, v)
        xd = x - d
        rxd, ryd = _residuals(xd, src, dst)
        Sd = lane_sum(rxd * rxd + ryd * ryd)
        temp = np.array([(A[i, 0] * d[0] + A[i, 1] * d[1] + A[i, 2] * d[2] + A[i, 3] * d[3]) * -1.0 + 2.0 * v[i]
                         for i in range(4)])  # gemm(A, d, -1, v, 2)
        dS = d[0] * temp[0] + d[1] * temp[1] + d[2] * temp[2] + d[3] * temp[3]
        R = (S - Sd) / (dS if abs(dS) > DBL_EPSILON else 1.0)
        if R > Rhi:
            lam *= 0.5
            if lam < lc:
                lam = 0.0
        elif R < Rlo:
            tt = d[0] * v[0] + d[1] * v[1] + d[2] * v[2] + d[3] * v[3]
            nu = (Sd - S) / (tt if abs(tt) > DBL_EPSILON else 1.0) + 2.0
            nu = min(max(nu, 2.0), 10.0)
            if lam == 0.0:
                lam = lc = 1.0 / _inv_diag_max(A)
                nu *= 0.5
            lam *= nu
        if Sd < S:
            S = Sd
            x = xd
            A, v, _, rinf = _normal(x, src, dst)
        it += 1
        dinf = float(np.max(np.abs(d)))
        if not (it < max_iters and dinf >= eps and rinf >= eps):
            break
    return x


def estimate_affine_partial_2d(frm, to):
    """cv2.estimateAffinePartial2D(frm, to, cv2.RANSAC) with its defaults: (H 2x3 float64 or None,
    inlier mask)."""
    frm = np.asarray(frm, np.float32).reshape(-1, 2)
    to = np.asarray(to, np.float32).reshape(-1, 2)
    M, mask, _ = ransac_partial_affine(frm, to)
    if M is None:
        return None, np.zeros(len(frm), np.uint8)
    if len(frm) > 2:
        keep = mask.astype(bool)  # compressElems: inliers first, in order
        src, dst = frm[keep], to[keep]
        if len(src):
            h = lm_refine(np.array([M[0, 0], M[1, 0], M[0, 2], M[1, 2]]), src, dst)
            M = np.array([[h[0], -h[1], h[2]], [h[1], h[0], h[3]]], np.float64)
    return M, mask


# ------------------------------------------------------------------ GMC
class RefGMC:
    """GMC(method='sparseOptFlow' | 'none', downscale=2) (gmc.py:48-105, 278-353)."""

    def __init__(self, method: str = "sparseOptFlow", downscale: int = 2):
        if method not in ("sparseOptFlow", "none", None):
            raise NotImplementedError(f"GMC method {method!r}: only sparseOptFlow / none are restated")
        self.method = method
        self.downscale = max(1, downscale)
        self.reset_params()
        self.last = {}

    def reset_params(self):
        self.prevFrame = None
        self.prevKeyPoints = None
        self.initializedFirstFrame = False

    def apply(self, raw_frame, detections=None):
        if self.method == "sparseOptFlow":
            return self.apply_sparseoptflow(raw_frame)
        return np.eye(2, 3)

    def apply_sparseoptflow(self, raw_frame):
        height, width, c = raw_frame.shape
        frame = G.bgr_to_gray(raw_frame) if c == 3 else raw_frame
        H = np.eye(2, 3)
        if self.downscale > 1:
            if self.downscale != 2 or (width % 2) or (height % 2):
                raise NotImplementedError("restated for downscale 2 of even frame sizes (INTER_AREA fast path)")
            frame = area_down2(frame)
        keypoints = G.good_features(frame, MAX_CORNERS, QUALITY, MIN_DIST, BLOCK)
        self.last = {"keypoints": keypoints}
        if not self.initializedFirstFrame or self.prevKeyPoints is None:
            self.prevFrame = frame.copy()
            self.prevKeyPoints = copy.copy(keypoints)
            self.initializedFirstFrame = True
            return H
        nxt, status = G.optical_flow(self.prevFrame, frame, self.prevKeyPoints)
        ok = status.astype(bool)
        prevPoints = self.prevKeyPoints.reshape(-1, 2)[ok]
        currPoints = nxt.reshape(-1, 2)[ok]
        self.last.update({"next": nxt, "status": status, "n_points": int(ok.sum())})
        if prevPoints.shape[0] > 4 and prevPoints.shape[0] == currPoints.shape[0]:
            M, inl = estimate_affine_partial_2d(prevPoints, currPoints)
            self.last["inliers"] = inl
            if M is None:
                # cv2 returns None: `H[0, 2] *= ...` raises before prevFrame / prevKeyPoints are
                # replaced, and BYTETracker.update's try (byte_tracker.py:334-338) uses np.eye(2, 3)
                self.last["failed"] = True
                return np.eye(2, 3)
            H = M
            if self.downscale > 1:
                H[0, 2] *= self.downscale
                H[1, 2] *= self.downscale
        self.prevFrame = frame.copy()
        self.prevKeyPoints = copy.copy(keypoints)
        return H
