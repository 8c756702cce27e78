"""TrajectoryVisualizer on the host (reference: kalman/trajectory_visualizer.py:5-235).

The reference draws with cv2 on the BGR frame the driver read (aircraft_detection_tracking.py:
143).  Drawing is output formatting, off the hot path ("drawing stays on the
host"), so this module works on the host copy of the frame in numpy.  cv2 is not installed in
this image, so the primitives restate OpenCV 4.x's published drawing algorithms
(modules/imgproc/src/drawing.cpp) where they are integer-exact and approximate them otherwise:

* ``line`` thickness 1 (LINE_8): ``clipLine`` followed by the 8-connected ``LineIterator``
  walk (left-to-right swap, ``err = dx - 2*dy`` error term) -- exact restatement.
* ``rectangle`` thickness 1: the closed 4-point polyline of 1-pixel lines -- exact; filled
  (thickness < 0): every pixel of ``[min x, max x] x [min y, max y]`` -- exact.
* thickness > 1 lines (``ThickLine``: a filled quad plus round caps in 16.16 fixed point):
  every pixel whose centre lies within ``thickness / 2`` of the segment -- approximate.
* ``arrowed_line``: OpenCV's ``arrowedLine`` geometry (tip length ``tipLength * |p1 - p2|``,
  wings at +-45 degrees, ``cvRound``) over the line above.
* ``add_weighted``: ``saturate_cast<uchar>(a * alpha + b * beta + gamma)`` in float32 with
  round-half-even (OpenCV's ``addWeighted`` 8U path).
* ``put_text`` / ``get_text_size``: the Hershey vector fonts are OpenCV-internal tables that are
  not in this image; text is rasterised with Pillow's bundled font, sized to the Hershey simplex
  cap height (21 units x ``font_scale``), anchored at the baseline like ``cv2.putText``;
  characters outside ASCII print as ``?`` as in OpenCV.  Approximate (layout, not glyph parity).

Parity with cv2 itself is unpinned (cv2 absent); ``tests/test_visualize_cpu.py`` pins the
integer-exact primitives against their restated definitions and the visualizer's status/colour
logic against the reference's.
"""
from __future__ import annotations

import math

import numpy as np

FONT_HERSHEY_SIMPLEX = 0
LINE_8 = 8


# ---------------------------------------------------------------------------------------------
# primitives
# ---------------------------------------------------------------------------------------------
def _check(img):
    if not isinstance(img, np.ndarray) or img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
        raise TypeError("image must be an HxWx3 uint8 (BGR) ndarray")


def clip_line(w: int, h: int, p1, p2):
    """OpenCV ``clipLine(Size, Point&, Point&)``: returns (inside, p1, p2)."""
    x1, y1 = int(p1[0]), int(p1[1])
    x2, y2 = int(p2[0]), int(p2[1])
    if w <= 0 or h <= 0:
        return False, (x1, y1), (x2, y2)
    right, bottom = w - 1, h - 1
    c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8
    c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8
    if (c1 & c2) == 0 and (c1 | c2) != 0:
        if c1 & 12:
            a = 0 if c1 < 8 else bottom
            x1 += int((a - y1) * (x2 - x1) / (y2 - y1))
            y1 = a
            c1 = (x1 < 0) + (x1 > right) * 2
        if c2 & 12:
            a = 0 if c2 < 8 else bottom
            x2 += int((a - y2) * (x2 - x1) / (y2 - y1))
            y2 = a
            c2 = (x2 < 0) + (x2 > right) * 2
        if (c1 & c2) == 0 and (c1 | c2) != 0:
            if c1:
                a = 0 if c1 == 1 else right
                y1 += int((a - x1) * (y2 - y1) / (x2 - x1))
                x1 = a
                c1 = 0
            if c2:
                a = 0 if c2 == 1 else right
                y2 += int((a - x2) * (y2 - y1) / (x2 - x1))
                x2 = a
                c2 = 0
    return (c1 | c2) == 0, (x1, y1), (x2, y2)


def line_pixels(w: int, h: int, p1, p2):
    """Pixels of a 1-pixel LINE_8 line in OpenCV's LineIterator order -> (xs, ys) int arrays."""
    ok, (x1, y1), (x2, y2) = clip_line(w, h, p1, p2)
    if not ok:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    if x2 < x1:  # leftToRight
        x1, y1, x2, y2 = x2, y2, x1, y1
    dx, dy = x2 - x1, y2 - y1
    sy = -1 if dy < 0 else 1
    dy = abs(dy)
    steep = dy > dx
    if steep:
        dx, dy = dy, dx
    err = dx - (dy + dy)
    plus, minus = dx + dx, -(dy + dy)
    n = dx + 1
    xs = np.empty(n, np.int64)
    ys = np.empty(n, np.int64)
    x, y = x1, y1
    for i in range(n):
        xs[i], ys[i] = x, y
        diag = err < 0
        err += minus + (plus if diag else 0)
        if steep:  # major axis y (the swapped pointer steps), minor x
            y += sy
            if diag:
                x += 1
        else:
            x += 1
            if diag:
                y += sy
    return xs, ys


def _capsule(img, p1, p2, color, thickness):
    h, w = img.shape[:2]
    r = thickness / 2.0
    x0 = max(int(math.floor(min(p1[0], p2[0]) - r)), 0)
    x1 = min(int(math.ceil(max(p1[0], p2[0]) + r)), w - 1)
    y0 = max(int(math.floor(min(p1[1], p2[1]) - r)), 0)
    y1 = min(int(math.ceil(max(p1[1], p2[1]) + r)), h - 1)
    if x0 > x1 or y0 > y1:
        return
    yy, xx = np.mgrid[y0:y1 + 1, x0:x1 + 1].astype(np.float64)
    ax, ay = float(p1[0]), float(p1[1])
    bx, by = float(p2[0]), float(p2[1])
    vx, vy = bx - ax, by - ay
    L2 = vx * vx + vy * vy
    t = np.zeros_like(xx) if L2 == 0 else np.clip(((xx - ax) * vx + (yy - ay) * vy) / L2, 0.0, 1.0)
    d2 = (xx - ax - t * vx) ** 2 + (yy - ay - t * vy) ** 2
    m = d2 <= r * r
    img[y0:y1 + 1, x0:x1 + 1][m] = color


def line(img, pt1, pt2, color, thickness: int = 1, lineType: int = LINE_8):
    """cv2.line (LINE_8)."""
    _check(img)
    color = np.asarray(color, np.uint8)[:3]
    if thickness <= 1:
        xs, ys = line_pixels(img.shape[1], img.shape[0], pt1, pt2)
        img[ys, xs] = color
    else:
        _capsule(img, pt1, pt2, color, int(thickness))
    return img


def rectangle(img, pt1, pt2, color, thickness: int = 1, lineType: int = LINE_8):
    """cv2.rectangle: closed polyline (thickness >= 0) or filled box (thickness < 0)."""
    _check(img)
    h, w = img.shape[:2]
    x1, y1 = int(pt1[0]), int(pt1[1])
    x2, y2 = int(pt2[0]), int(pt2[1])
    if thickness < 0:
        xa, xb = max(min(x1, x2), 0), min(max(x1, x2), w - 1)
        ya, yb = max(min(y1, y2), 0), min(max(y1, y2), h - 1)
        if xa <= xb and ya <= yb:
            img[ya:yb + 1, xa:xb + 1] = np.asarray(color, np.uint8)[:3]
        return img
    pts = [(x1, y1), (x2, y1), (x2, y2), (x1, y2)]
    for i in range(4):
        line(img, pts[i], pts[(i + 1) % 4], color, thickness)
    return img


def _cv_round(v: float) -> int:
    return int(np.rint(v))


def arrowed_line(img, pt1, pt2, color, thickness: int = 1, tipLength: float = 0.1):
    """cv2.arrowedLine: the shaft plus two wings of length tipLength * |pt1 - pt2| at +-45 deg."""
    line(img, pt1, pt2, color, thickness)
    angle = math.atan2(pt1[1] - pt2[1], pt1[0] - pt2[0])
    tip = math.hypot(pt1[0] - pt2[0], pt1[1] - pt2[1]) * tipLength
    for s in (1, -1):
        p = (_cv_round(pt2[0] + tip * math.cos(angle + s * math.pi / 4)),
             _cv_round(pt2[1] + tip * math.sin(angle + s * math.pi / 4)))
        line(img, p, pt2, color, thickness)
    return img


def add_weighted(src1, alpha, src2, beta, gamma, dst=None):
    """cv2.addWeighted for uint8: saturate(round_half_even(a*alpha + b*beta + gamma)) in float32."""
    a = src1.astype(np.float32) * np.float32(alpha)
    b = src2.astype(np.float32) * np.float32(beta)
    r = np.clip(np.rint(a + b + np.float32(gamma)), 0, 255).astype(np.uint8)
    if dst is not None:
        dst[...] = r
        return dst
    return r


# -- text ---------------------------------------------------------------------------------------
_FONTS = {}


def _font(px: int):
    f = _FONTS.get(px)
    if f is None:
        try:
            from PIL import ImageFont
        except ImportError as e:  # text needs a rasteriser; boxes/lines/trails do not
            raise RuntimeError("put_text needs Pillow (cv2's Hershey fonts are not in this image)") from e
        f = ImageFont.load_default(size=max(px, 4))
        _FONTS[px] = f
    return f


def _ascii(text: str) -> str:
    return "".join(c if 32 <= ord(c) < 127 else "?" for c in str(text))


def _cap_px(font_scale: float) -> int:
    return max(int(round(21 * float(font_scale))), 4)  # Hershey simplex cap height: 21 units


def get_text_size(text, fontFace=FONT_HERSHEY_SIMPLEX, fontScale=1.0, thickness=1):
    """((width, height), baseline) like cv2.getTextSize, from the rasterised text."""
    t = _ascii(text)
    cap = _cap_px(fontScale)
    f = _font(int(round(cap / 0.72)))
    x0, y0, x1, y1 = f.getbbox(t or " ", anchor="ls")
    extra = (int(thickness) + 1) // 2
    return (max(x1 - x0, 0) + extra, cap + extra), max(y1, 0) + extra


def put_text(img, text, org, fontFace, fontScale, color, thickness=1, lineType=LINE_8):
    """cv2.putText: ``org`` is the left end of the baseline."""
    _check(img)
    from PIL import Image, ImageDraw

    t = _ascii(text)
    if not t:
        return img
    cap = _cap_px(fontScale)
    f = _font(int(round(cap / 0.72)))
    x0, y0, x1, y1 = f.getbbox(t, anchor="ls")
    pad = int(thickness)
    W, H = x1 - x0 + 2 * pad + 2, y1 - y0 + 2 * pad + 2
    mask = Image.new("L", (W, H), 0)
    ImageDraw.Draw(mask).text((pad - x0 + 1, pad - y0 + 1), t, fill=255, font=f, anchor="ls")
    m = np.asarray(mask) >= 128
    for _ in range(max(int(thickness) - 1, 0)):  # thicker strokes: dilate by one pixel per step
        d = m.copy()
        d[1:] |= m[:-1]
        d[:-1] |= m[1:]
        d[:, 1:] |= m[:, :-1]
        d[:, :-1] |= m[:, 1:]
        m = d
    ox, oy = int(org[0]) + x0 - pad - 1, int(org[1]) + y0 - pad - 1
    h, w = img.shape[:2]
    ya, yb = max(oy, 0), min(oy + H, h)
    xa, xb = max(ox, 0), min(ox + W, w)
    if ya < yb and xa < xb:
        sub = m[ya - oy:yb - oy, xa - ox:xb - ox]
        img[ya:yb, xa:xb][sub] = np.asarray(color, np.uint8)[:3]
    return img


# ---------------------------------------------------------------------------------------------
# the reference's visualizer
# ---------------------------------------------------------------------------------------------
class TrajectoryVisualizer:
    """kalman/trajectory_visualizer.py:5-235 on numpy BGR frames (same colours, layout and
    status logic; ``draw_tracks`` returns a new frame and leaves the input untouched)."""

    def __init__(self, colors=None):
        self.colors = colors or {
            "detected": (0, 255, 0),
            "predicted": (0, 165, 255),
            "lost": (0, 100, 255),
            "trajectory": (255, 255, 0),
            "velocity": (255, 0, 255),
            "text": (255, 255, 255),
            "background": (0, 0, 0),
        }
        self.trajectory_length = 20
        self.velocity_scale = 5.0
        self.font = FONT_HERSHEY_SIMPLEX
        self.font_scale = 0.4
        self.font_thickness = 1
        self.frame_counter = 0

    def draw_tracks(self, image, tracks, detections=None, frame_info=None):  # :29-44
        vis = np.array(image, dtype=np.uint8, copy=True)
        self.frame_counter += 1
        if detections:
            self._draw_detections(vis, detections)
        for t in tracks:
            self._draw_single_track(vis, t)
        if frame_info:
            self._draw_frame_info(vis, frame_info, tracks, detections)
        self._draw_legend(vis)
        return vis

    def _draw_detections(self, image, detections):  # :46-54
        for det in detections:
            if len(det) >= 5:
                x1, y1, x2, y2, conf = det[:5]
                x1, y1, x2, y2 = map(int, [x1, y1, x2, y2])
                rectangle(image, (x1, y1), (x2, y2), self.colors["detected"], 1)
                put_text(image, f"Det: {conf:.2f}", (x1, y1 - 5), self.font, 0.3, self.colors["detected"], 1)

    def flash(self):
        """Colour and thickness of a predicted box this frame (:68-75: 6-frame flash cycle)."""
        if (self.frame_counter // 6) % 2 == 0:
            return (0, 220, 255), 2
        return self.colors["predicted"], 1

    def _draw_single_track(self, image, track):  # :56-117
        bbox = track["bbox"]
        track_id = str(track["track_id"])
        status = track.get("status", "detected")
        tsu = int(track.get("time_since_update", 0))
        confidence = float(track.get("confidence", 1.0))
        trajectory = track.get("trajectory", [])
        velocity = track.get("velocity", (0, 0))
        x1, y1, x2, y2 = [int(float(c)) for c in bbox[:4]]
        if status == "predicted":
            color, thickness = self.flash()
            rectangle(image, (x1, y1), (x2, y2), color, thickness)
            overlay = image.copy()
            rectangle(overlay, (x1, y1), (x2, y2), color, -1)
            add_weighted(overlay, 0.3, image, 0.7, 0, image)
            self._draw_label(image, f"ID:{track_id} PRED({tsu})", x1, y1, x2, y2, color)
            self._draw_status_text(image, "⚠️ AI PREDICTION", x2, y1, color)
        else:
            color = self.colors["detected"]
            rectangle(image, (x1, y1), (x2, y2), color, 1)
            self._draw_label(image, f"ID:{track_id} TRACKING", x1, y1, x2, y2, color)
            self._draw_status_text(image, "✅ DETECTED", x2, y1, color)
        put_text(image, f"Conf: {confidence:.2f}", (x2 + 10, y2 + 10), self.font, 0.3, self.colors["text"], 1)
        color = self.colors["predicted"] if status == "predicted" else self.colors["detected"]
        self._draw_trajectory(image, trajectory, color)
        vx, vy = velocity
        if np.sqrt(vx ** 2 + vy ** 2) > 1.0:
            self._draw_velocity_vector(image, bbox, velocity)

    def _draw_label(self, image, label, x1, y1, x2, y2, color):  # :119-135
        (tw, th), _ = get_text_size(label, self.font, self.font_scale, self.font_thickness)
        lx, ly = x2 + 15, y1 - 5
        rectangle(image, (lx - 2, ly - th - 2), (lx + tw + 2, ly + 2), color, -1)
        put_text(image, label, (lx, ly), self.font, self.font_scale, self.colors["text"], self.font_thickness)

    def _draw_status_text(self, image, text, x2, y1, color):  # :137-158
        (tw, th), _ = get_text_size(text, self.font, 0.35, 1)
        tx, ty = x2 + 20, y1 + 15
        h, w = image.shape[:2]
        if tx + tw > w:
            tx = x2 - tw - 20
        if ty > h:
            ty = y1 - 10
        rectangle(image, (tx - 2, ty - th - 2), (tx + tw + 2, ty + 2), color, -1)
        put_text(image, text, (tx, ty), self.font, 0.35, (255, 255, 255), 1)

    def _draw_trajectory(self, image, trajectory, color):  # :160-172 (trail colour is 'trajectory')
        if len(trajectory) < 2:
            return
        pts = np.array(list(trajectory)[-self.trajectory_length:], dtype=np.float64).astype(np.int32)
        for i in range(1, len(pts)):
            alpha = i / len(pts)
            line(image, tuple(pts[i - 1]), tuple(pts[i]), self.colors["trajectory"], max(1, int(3 * alpha)))

    def _draw_velocity_vector(self, image, bbox, velocity):  # :174-184
        cx = int((bbox[0] + bbox[2]) / 2)
        cy = int((bbox[1] + bbox[3]) / 2)
        vx, vy = velocity
        ex = int(cx + vx * self.velocity_scale)
        ey = int(cy + vy * self.velocity_scale)
        arrowed_line(image, (cx, cy), (ex, ey), self.colors["velocity"], 2, tipLength=0.3)

    def _draw_frame_info(self, image, frame_info, tracks, detections):  # :186-208
        det_n = sum(1 for t in tracks if t.get("status") == "detected")
        pred_n = sum(1 for t in tracks if t.get("status") == "predicted")
        texts = [
            f"Frame: {frame_info.get('frame_number', 0)}",
            f"Detections: {len(detections) if detections else 0}",
            f"Tracking (Green): {det_n}",
            f"Predicting (Orange): {pred_n}",
        ]
        if "state_changes" in frame_info:
            texts.append(f"State Changes: {frame_info['state_changes']}")
        for i, t in enumerate(texts):
            put_text(image, t, (10, 30 + i * 25), self.font, 0.6, self.colors["text"], 2)

    def _draw_legend(self, image):  # :210-234
        h, w = image.shape[:2]
        lx, ly = w - 220, h - 100
        rectangle(image, (lx - 10, ly - 10), (w - 10, h - 10), self.colors["background"], -1)
        rectangle(image, (lx - 10, ly - 10), (w - 10, h - 10), self.colors["text"], 2)
        put_text(image, "Status Legend", (lx, ly - 5), self.font, 0.6, self.colors["text"], 2)
        legends = [("Green = Detection", self.colors["detected"]),
                   ("Orange = Prediction", self.colors["predicted"]),
                   ("Yellow = Trail", self.colors["trajectory"])]
        for i, (label, color) in enumerate(legends):
            y = ly + 15 + i * 20
            rectangle(image, (lx, y), (lx + 15, y + 15), color, -1)
            put_text(image, label, (lx + 25, y + 12), self.font, 0.45, self.colors["text"], 1)
