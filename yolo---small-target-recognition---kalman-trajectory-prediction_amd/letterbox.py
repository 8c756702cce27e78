"""LetterBox geometry and the resize tables of the device letterbox kernel.

Reference: ultralytics/data/augment.py:1667-1744 (LetterBox.__call__ with auto=True,
center=True, padding 114) calling cv2.resize(img, new_unpad, INTER_LINEAR) when the frame is not
already at the network size, and utils/ops.py:105-184 (scale_boxes + clip_boxes) mapping the
boxes back.  cv2.resize is a third-party dependency absent here; the kernel restates OpenCV
4.x's 8-bit INTER_LINEAR path (imgproc/src/resize.cpp):

  * an exact 2x downscale in both axes is routed to INTER_AREA's fast path:
    dst = (a + b + c + d + 2) >> 2 over the 2x2 source block;
  * otherwise per destination column: fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor(fx),
    fx -= sx, clamped at both borders to (sx, fx) = (0, 0) / (w - 1, 0); fixed-point weights
    saturate_cast<short>((1 - fx) * 2048), saturate_cast<short>(fx * 2048) (round half even);
    the same per destination row; horizontal pass D = S[sx] * a0 + S[sx + 1] * a1 (int32);
    rows are not clamped: the fetch clips sy and sy + 1 into the image, both weights kept;
    vertical pass with the 128-bit SIMD rounding ((((D0 >> 4) * b0) >> 16) + (((D1 >> 4) * b1)
    >> 16) + 2) >> 2 on the elements the vector loops cover (rows of W*3 bytes: 16-byte blocks,
    then 8-byte blocks while x < W*3 - 8) and the scalar (D0 * b0 + D1 * b1 + 2^21) >> 22 on the
    rest.
Parity with cv2 itself is unpinned (no cv2 in this environment); the oracle
(oracle/letterbox_ref.py) restates the same published algorithm independently.
"""
from __future__ import annotations

import math

import numpy as np

RS_NONE, RS_LINEAR, RS_AREA2 = 0, 1, 2
COEF_SCALE = 2048  # INTER_RESIZE_COEF_SCALE


def _coeffs(dst: int, src: int, clamp: bool):
    """Per destination index: source index and the two fixed-point weights.  Columns are
    clamped at the borders (sx, fx) -> (0, 0) / (w - 1, 0); rows are not (the row fetch clips
    sy and sy + 1 into the image instead, keeping both weights)."""
    scale = 1.0 / (dst / src)  # scale_x = 1. / inv_scale_x
    ofs = np.zeros(dst, np.int32)
    w = np.zeros((dst, 2), np.int16)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if clamp and s < 0:
            s, f = 0, np.float32(0)
        if clamp and s + 1 >= src:
            s, f = src - 1, np.float32(0)
        c0 = np.float32(np.float32(1.0) - f) * np.float32(COEF_SCALE)
        c1 = f * np.float32(COEF_SCALE)
        ofs[d] = s
        w[d] = (int(np.clip(np.rint(c0), -32768, 32767)), int(np.clip(np.rint(c1), -32768, 32767)))
    return ofs, w


def plan(frame_h: int, frame_w: int, imgsz=640, stride: int = 32) -> dict:
    if isinstance(imgsz, int):
        imgsz = (imgsz, imgsz)
    r = min(imgsz[0] / frame_h, imgsz[1] / frame_w)
    new_w, new_h = int(round(frame_w * r)), int(round(frame_h * r))
    dw, dh = (imgsz[1] - new_w) % stride, (imgsz[0] - new_h) % stride
    dw, dh = dw / 2, dh / 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    in_h, in_w = new_h + top + bottom, new_w + left + right
    out = dict(in_h=in_h, in_w=in_w, top=top, left=left, new_h=new_h, new_w=new_w, mode=RS_NONE)
    if (new_w, new_h) != (frame_w, frame_h):
        sx, sy = 1.0 / (new_w / frame_w), 1.0 / (new_h / frame_h)
        if abs(sx - round(sx)) < np.finfo(float).eps and abs(sy - round(sy)) < np.finfo(float).eps \
                and round(sx) == 2 and round(sy) == 2:
            out["mode"] = RS_AREA2
        else:
            out["mode"] = RS_LINEAR
        out["xofs"], out["xw"] = _coeffs(new_w, frame_w, True)
        out["yofs"], out["yw"] = _coeffs(new_h, frame_h, False)
    # scale_boxes (ops.py:123-126): gain and padding recomputed from the two shapes
    gain = min(in_h / frame_h, in_w / frame_w)
    out["gain"] = gain
    out["pad_x"] = round((in_w - frame_w * gain) / 2 - 0.1)
    out["pad_y"] = round((in_h - frame_h * gain) / 2 - 0.1)
    return out


def table_blob(p: dict) -> np.ndarray:
    """int32 [xofs (new_w) | yofs (new_h) | xw (new_w x 2 int16 packed) | yw (new_h x 2 int16 packed)]."""
    if p["mode"] == RS_NONE:
        return np.zeros(4, np.int32)
    xw = p["xw"].view(np.int32).reshape(-1)
    yw = p["yw"].view(np.int32).reshape(-1)
    return np.concatenate([p["xofs"], p["yofs"], xw, yw]).astype(np.int32)
