"""numpy restatement of LetterBox's resize (TEST ORACLE ONLY).

ultralytics/data/augment.py:1717-1719 calls cv2.resize(img, new_unpad, INTER_LINEAR); cv2 is a
third-party dependency absent from this environment (no opencv wheel), so this file restates
OpenCV 4.x's published 8-bit algorithm (imgproc/src/resize.cpp: cv::resize -> hal::resize,
resizeAreaFast_Invoker, resizeGeneric_ with HResizeLinear / VResizeLinear and
VResizeLinearVec_32s8u under 128-bit universal intrinsics).  Parity with cv2 itself is
unpinned: there is no fixture in the reference that holds a resized image.

  * scale exactly 2 in both axes -> INTER_AREA fast path, (a + b + c + d + 2) >> 2;
  * else fixed-point bilinear: per axis fx = float32((d + 0.5) * scale - 0.5), s = floor(fx),
    fx -= s; columns clamped to (0, 0) / (w - 1, 0), rows unclamped with the fetch clipped;
    weights rint((1 - fx) * 2048), rint(fx * 2048) (round half even); horizontal int32 sums;
    vertical rounding of the SIMD loops on the first `vec_end` bytes of a row, scalar beyond.
"""
from __future__ import annotations

import numpy as np


def _axis(dst: int, src: int, clamp: bool):
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * (1.0 / (dst / src)) - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp:
        lo = s < 0
        s[lo], f[lo] = 0, 0
        hi = s + 1 >= src
        s[hi], f[hi] = src - 1, 0
    w0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    w1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return s, w0, w1


def resize_linear(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h), interpolation=INTER_LINEAR) for uint8 HxWx3."""
    h, w, cn = img.shape
    sx, sy = 1.0 / (new_w / w), 1.0 / (new_h / h)
    eps = np.finfo(np.float64).eps
    if abs(sx - round(sx)) < eps and abs(sy - round(sy)) < eps and round(sx) == 2 and round(sy) == 2:
        a = img[0:2 * new_h:2, 0:2 * new_w:2].astype(np.int64)
        b = img[0:2 * new_h:2, 1:2 * new_w:2].astype(np.int64)
        c = img[1:2 * new_h:2, 0:2 * new_w:2].astype(np.int64)
        d = img[1:2 * new_h:2, 1:2 * new_w:2].astype(np.int64)
        return ((a + b + c + d + 2) >> 2).astype(np.uint8)
    xs, xa0, xa1 = _axis(new_w, w, True)
    ys, yb0, yb1 = _axis(new_h, h, False)
    xs1 = np.minimum(xs + 1, w - 1)
    src = img.astype(np.int64)
    horiz = src[:, xs, :] * xa0[None, :, None] + src[:, xs1, :] * xa1[None, :, None]  # [h, new_w, cn]
    r0 = np.clip(ys, 0, h - 1)
    r1 = np.clip(ys + 1, 0, h - 1)
    d0, d1 = horiz[r0], horiz[r1]                      # [new_h, new_w, cn]
    b0, b1 = yb0[:, None, None], yb1[:, None, None]
    # SIMD path: int16 (D >> 4), mul_hi (>> 16, arithmetic), sum, (+2) >> 2
    simd = ((((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16) + 2) >> 2
    scal = (d0 * b0 + d1 * b1 + (1 << 21)) >> 22
    W = new_w * cn
    xv = W // 16 * 16 if W >= 16 else 0
    while xv < W - 8:
        xv += 8
    elem = (np.arange(new_w)[:, None] * cn + np.arange(cn)[None, :])[None]  # [1, new_w, cn]
    out = np.where(elem < xv, simd, scal)
    return np.clip(out, 0, 255).astype(np.uint8)


def letterbox(img: np.ndarray, imgsz=640, stride=32, pad_value=114):
    """LetterBox(auto=True, center=True)(image=img) -> the padded uint8 canvas
    (data/augment.py:1690-1729)."""
    h, w = img.shape[:2]
    r = min(imgsz / h, imgsz / w)
    new_w, new_h = int(round(w * r)), int(round(h * r))
    dw, dh = (imgsz - new_w) % stride / 2, (imgsz - new_h) % stride / 2
    if (w, h) != (new_w, new_h):
        img = resize_linear(img, new_w, new_h)
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return np.pad(img, ((top, bottom), (left, right), (0, 0)), constant_values=pad_value)
