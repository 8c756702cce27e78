"""Frame sources and sinks for the predict path (reference: data/loaders.py:309-563,
utils/patches.py:20-47, and the driver's cv2.VideoCapture / VideoWriter loop,
kalman/aircraft_detection_tracking.py:58-73,88-89,161).

The detector consumes ``HxWx3 uint8 BGR`` frames (what ``cv2.imread`` / ``VideoCapture.read``
return).  This module turns the sources ``YOLO.predict`` accepts into such frames, on the host,
before they are copied into HBM:

* ``numpy`` arrays (``LoadPilAndNumpy``, loaders.py:492-563): an HxWx3 frame, an HxW grey frame
  (expanded to 3 channels), or an NxHxWx3 stack; ``PIL.Image`` objects are converted to RGB
  and flipped to BGR exactly as ``_single_check`` does (loaders.py:537-547);
* image files, directories and glob patterns (``LoadImagesAndVideos``, loaders.py:309-490, the
  suffixes of data/utils.py:39): decoded with Pillow to RGB, then flipped to BGR.  For lossless
  formats (png, bmp, tif, pfm) this is the same array ``cv2.imread`` returns; JPEG decoders
  differ between libjpeg builds, so jpg/webp pixels are decoder-dependent in the reference too;
* ``.npy`` files: an HxWx3 frame or an NxHxWx3 frame stack (a raw "video"; loaded with
  ``allow_pickle=False``).

Compressed video (mp4/avi/...) needs a codec; neither cv2 nor ffmpeg is in this image, so
``VideoReader`` reads frame stacks (``.npy``), image directories / globs and YUV4MPEG2 (``.y4m``,
4:4:4 or 4:2:0 8-bit, converted with OpenCV's BT.601 ``COLOR_YUV2BGR`` integer coefficients)
and raises ``NotImplementedError`` naming the missing codec for anything else.
``VideoWriter`` writes the same containers (``.npy`` stack, or numbered PNGs into a directory).
"""
from __future__ import annotations

import glob as _glob
import os

import numpy as np

IMG_FORMATS = {"bmp", "dng", "jpeg", "jpg", "mpo", "png", "tif", "tiff", "webp", "pfm", "heic"}
VID_FORMATS = {"asf", "avi", "gif", "m4v", "mkv", "mov", "mp4", "mpeg", "mpg", "ts", "wmv", "webm"}

CAP_PROP_FPS = 5
CAP_PROP_FRAME_WIDTH = 3
CAP_PROP_FRAME_HEIGHT = 4
CAP_PROP_FRAME_COUNT = 7
CAP_PROP_POS_FRAMES = 1


def _suffix(p: str) -> str:
    return os.path.splitext(str(p))[1][1:].lower()


def _as_bgr(a: np.ndarray) -> np.ndarray:
    if a.dtype != np.uint8:
        raise ValueError(f"frames must be uint8, got {a.dtype}")
    if a.ndim == 2:  # grey: LoadPilAndNumpy adds the channel axis; cv2 IMREAD_COLOR replicates it
        a = np.repeat(a[:, :, None], 3, axis=2)
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"expected an HxWx3 BGR frame, got shape {a.shape}")
    return np.ascontiguousarray(a)


def pil_to_bgr(im) -> np.ndarray:
    """loaders.py:537-547: ``np.asarray(im.convert('RGB'))[..., ::-1]``."""
    return np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])


def imread(path: str) -> np.ndarray:
    """patches.py:20-47 ``imread(path, IMREAD_COLOR)`` -> HxWx3 BGR uint8 (Pillow decode)."""
    sfx = _suffix(path)
    if sfx == "npy":
        return _as_bgr(np.load(path, allow_pickle=False))
    if sfx not in IMG_FORMATS:
        raise ValueError(f"{path}: not an image file (suffixes {sorted(IMG_FORMATS)})")
    try:
        from PIL import Image
    except ImportError as e:
        raise RuntimeError("decoding image files needs Pillow (cv2 is not in this image)") from e
    with Image.open(path) as im:
        return pil_to_bgr(im)


def imwrite(path: str, frame: np.ndarray) -> None:
    from PIL import Image

    Image.fromarray(np.ascontiguousarray(_as_bgr(frame)[:, :, ::-1])).save(path)


def _expand_paths(p: str):
    p = str(p)
    if any(c in p for c in "*?["):
        files = sorted(_glob.glob(p, recursive=True))
    elif os.path.isdir(p):
        files = sorted(os.path.join(p, f) for f in os.listdir(p))
    elif os.path.isfile(p):
        files = [p]
    else:
        raise FileNotFoundError(f"{p} does not exist")
    return [f for f in files if _suffix(f) in IMG_FORMATS | VID_FORMATS | {"npy", "y4m"}]


def load_source(source):
    """Source (as YOLO.predict accepts it) -> list of (path, HxWx3 BGR uint8 frame)."""
    if isinstance(source, np.ndarray):
        if source.ndim == 4:
            return [(f"image{i}.jpg", _as_bgr(f)) for i, f in enumerate(source)]
        return [("image0.jpg", _as_bgr(source))]
    if isinstance(source, (list, tuple)):
        out = []
        for s in source:
            named = isinstance(s, (str, os.PathLike))
            out.extend((p if named else None, f) for p, f in load_source(s))
        # in-memory frames are named image{i}.jpg by their position in the batch, as the reference's
        # LoadPilAndNumpy does (loaders.py:528); files keep their paths
        return [(p if p is not None else f"image{i}.jpg", f) for i, (p, f) in enumerate(out)]
    if isinstance(source, (str, os.PathLike)):
        out = []
        for f in _expand_paths(source):
            sfx = _suffix(f)
            if sfx in IMG_FORMATS:
                out.append((f, imread(f)))
            else:  # frame stacks / videos: every frame, as LoadImagesAndVideos yields them
                with VideoReader(f) as cap:
                    i = 0
                    while True:
                        ok, fr = cap.read()
                        if not ok:
                            break
                        out.append((f"{f}:{i}", fr))
                        i += 1
        return out
    try:
        from PIL import Image

        if isinstance(source, Image.Image):
            return [("image0.jpg", pil_to_bgr(source))]
    except ImportError:
        pass
    raise TypeError(f"unsupported source type {type(source).__name__}: ndarray, PIL.Image, path, directory, "
                    "glob or a list of these")


# ---------------------------------------------------------------------------------------------
# video containers
# ---------------------------------------------------------------------------------------------
def _yuv2bgr(y, u, v):
    """OpenCV COLOR_YUV2BGR (BT.601 full range, 14-bit fixed point as in color_yuv.simd.hpp)."""
    yi = y.astype(np.int32)
    ui = u.astype(np.int32) - 128
    vi = v.astype(np.int32) - 128
    sh, half = 14, 1 << 13
    b = yi + ((ui * 33292 + half) >> sh)
    g = yi + ((ui * -6472 + vi * -9519 + half) >> sh)
    r = yi + ((vi * 18678 + half) >> sh)
    return np.clip(np.stack([b, g, r], axis=2), 0, 255).astype(np.uint8)


def _yuv420_to_bgr(y, u, v):
    """OpenCV COLOR_YUV2BGR_I420 (color_yuv.simd.hpp: BT.601 limited range, ITUR_BT_601_*
    constants, 20-bit fixed point, Y - 16 clamped at 0) on chroma already upsampled by 2x2
    replication, which is how that conversion shares one (u, v) pair per 2x2 block.  The
    reference driver's cv2.VideoCapture decodes through FFmpeg's own converter, whose rounding
    may differ in the last unit: parity with it is unpinned (no codec or cv2 in this image)."""
    cy, cub, cug, cvg, cvr, sh = 1220542, 2116026, -409993, -852492, 1673527, 20
    half = 1 << (sh - 1)
    yy = np.maximum(y.astype(np.int64) - 16, 0) * cy
    ui = u.astype(np.int64) - 128
    vi = v.astype(np.int64) - 128
    b = (yy + half + cub * ui) >> sh
    g = (yy + half + cvg * vi + cug * ui) >> sh
    r = (yy + half + cvr * vi) >> sh
    return np.clip(np.stack([b, g, r], axis=2), 0, 255).astype(np.uint8)


class VideoReader:
    """cv2.VideoCapture-like reader: ``read() -> (ok, frame)``, ``get(prop)``, ``isOpened()``."""

    def __init__(self, path, fps: float = 30.0):
        self.path = str(path)
        self._fps = float(fps)
        self._pos = 0
        self._frames = None
        self._files = None
        self._y4m = None
        sfx = _suffix(self.path)
        if os.path.isdir(self.path) or any(c in self.path for c in "*?["):
            self._files = [f for f in _expand_paths(self.path) if _suffix(f) in IMG_FORMATS]
            first = imread(self._files[0]) if self._files else None
            self._shape = None if first is None else first.shape
            self._n = len(self._files)
        elif sfx == "npy":
            a = np.load(self.path, allow_pickle=False, mmap_mode="r")
            if a.ndim == 3:
                a = a[None]
            if a.ndim != 4 or a.shape[3] != 3 or a.dtype != np.uint8:
                raise ValueError(f"{self.path}: expected an NxHxWx3 uint8 frame stack, got {a.shape} {a.dtype}")
            self._frames, self._shape, self._n = a, a.shape[1:], a.shape[0]
        elif sfx == "y4m":
            self._open_y4m()
        elif sfx in VID_FORMATS:
            raise NotImplementedError(f"{self.path}: decoding .{sfx} needs a video codec (cv2/ffmpeg), which this "
                                      "image does not have; convert the video to a .npy frame stack, an image "
                                      "directory or .y4m")
        else:
            raise ValueError(f"{self.path}: unsupported video container")

    def _open_y4m(self):
        f = open(self.path, "rb")
        header = f.readline().decode("ascii").split()
        if not header or header[0] != "YUV4MPEG2":
            raise ValueError(f"{self.path}: not a YUV4MPEG2 file")
        w = h = None
        chroma = "420jpeg"
        for tok in header[1:]:
            if tok[0] == "W":
                w = int(tok[1:])
            elif tok[0] == "H":
                h = int(tok[1:])
            elif tok[0] == "F":
                num, den = tok[1:].split(":")
                self._fps = float(num) / float(den)
            elif tok[0] == "C":
                chroma = tok[1:]
        if chroma.startswith("444"):
            csz = (h, w)
        elif chroma.startswith("420"):
            csz = ((h + 1) // 2, (w + 1) // 2)
        else:
            raise NotImplementedError(f"{self.path}: y4m chroma {chroma}")
        self._y4m = (f, w, h, csz, f.tell())
        fsz = len(b"FRAME\n") + w * h + 2 * csz[0] * csz[1]
        self._n = (os.path.getsize(self.path) - f.tell()) // fsz
        self._shape = (h, w, 3)

    def isOpened(self) -> bool:
        return self._n > 0 or self._files is not None

    def get(self, prop: int) -> float:
        if prop == CAP_PROP_FPS:
            return self._fps
        if prop == CAP_PROP_FRAME_WIDTH:
            return float(self._shape[1]) if self._shape else 0.0
        if prop == CAP_PROP_FRAME_HEIGHT:
            return float(self._shape[0]) if self._shape else 0.0
        if prop == CAP_PROP_FRAME_COUNT:
            return float(self._n)
        if prop == CAP_PROP_POS_FRAMES:
            return float(self._pos)
        return 0.0

    def read(self):
        if self._pos >= self._n:
            return False, None
        i = self._pos
        self._pos += 1
        if self._frames is not None:
            return True, np.array(self._frames[i])
        if self._files is not None:
            return True, imread(self._files[i])
        f, w, h, (ch, cw), _ = self._y4m
        line = f.readline()
        if not line.startswith(b"FRAME"):
            return False, None
        y = np.frombuffer(f.read(w * h), np.uint8).reshape(h, w)
        u = np.frombuffer(f.read(ch * cw), np.uint8).reshape(ch, cw)
        v = np.frombuffer(f.read(ch * cw), np.uint8).reshape(ch, cw)
        if (ch, cw) != (h, w):  # 4:2:0: OpenCV's I420 path (limited range), 2x2 chroma blocks
            u = np.repeat(np.repeat(u, 2, 0), 2, 1)[:h, :w]
            v = np.repeat(np.repeat(v, 2, 0), 2, 1)[:h, :w]
            return True, _yuv420_to_bgr(y, u, v)
        return True, _yuv2bgr(y, u, v)  # 4:4:4

    def release(self):
        if self._y4m is not None:
            self._y4m[0].close()
            self._y4m = None
        self._n = 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()

    def __iter__(self):
        while True:
            ok, fr = self.read()
            if not ok:
                return
            yield fr


class VideoWriter:
    """cv2.VideoWriter-like sink: ``.npy`` (one NxHxWx3 stack written on release) or a directory
    (``frame_000001.png`` ...).  Compressed containers need a codec this image does not have."""

    def __init__(self, path, fps: float = 30.0, frame_size=None):
        self.path = str(path)
        self.fps = float(fps)
        self.frame_size = tuple(frame_size) if frame_size is not None else None
        self._frames = []
        self._count = 0
        sfx = _suffix(self.path)
        if sfx == "npy":
            self._mode = "npy"
        elif sfx == "" or os.path.isdir(self.path):
            self._mode = "dir"
            os.makedirs(self.path, exist_ok=True)
        elif sfx in VID_FORMATS:
            raise NotImplementedError(f"{self.path}: encoding .{sfx} needs a video codec (cv2/ffmpeg), which this "
                                      "image does not have; write a .npy stack or a directory of PNGs")
        else:
            raise ValueError(f"{self.path}: unsupported output container")

    def isOpened(self) -> bool:
        return True

    def write(self, frame):
        fr = _as_bgr(np.asarray(frame))
        if self.frame_size is not None and (fr.shape[1], fr.shape[0]) != self.frame_size:
            return  # cv2.VideoWriter drops frames of the wrong size
        self._count += 1
        if self._mode == "npy":
            self._frames.append(fr.copy())
        else:
            imwrite(os.path.join(self.path, f"frame_{self._count:06d}.png"), fr)

    def release(self):
        if self._mode == "npy" and self._frames:
            np.save(self.path, np.stack(self._frames))
            self._frames = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()
