"""Host-side visualizer and frame I/O (SURVEY §8f-3 remainder; kalman/trajectory_visualizer.py,
data/loaders.py).  CPU only: no GPU and no oracle involved (drawing is host formatting).

cv2 is absent, so the OpenCV primitives are pinned against hand-derived runs of OpenCV's published
algorithms (LineIterator's error term, clipLine, rectangle's polyline, addWeighted's float32
rounding); parity with cv2 itself is unpinned."""
import importlib
import os

import numpy as np
import pytest

from conftest import PKG_NAME


def pkg_module(name):
    return importlib.import_module(f"{PKG_NAME}.{name}")


V = pkg_module("visualize")
FR = pkg_module("frames")


def test_line_iterator_kat():
    # LineIterator (connectivity 8) from (0,0) to (5,2): err = dx - 2dy = 1, steps by hand
    xs, ys = V.line_pixels(20, 20, (0, 0), (5, 2))
    assert list(zip(xs, ys)) == [(0, 0), (1, 0), (2, 1), (3, 1), (4, 2), (5, 2)]
    # left-to-right swap: the same pixel set when given backwards
    xs2, ys2 = V.line_pixels(20, 20, (5, 2), (0, 0))
    assert list(zip(xs2, ys2)) == list(zip(xs, ys))
    # steep line: y is the major axis
    xs, ys = V.line_pixels(20, 20, (0, 0), (2, 5))
    assert list(zip(xs, ys)) == [(0, 0), (0, 1), (1, 2), (1, 3), (2, 4), (2, 5)]


@pytest.mark.parametrize("p1,p2", [((3, 4), (17, 9)), ((1, 18), (12, 0)), ((7, 7), (7, 19)), ((0, 5), (19, 5))])
def test_line_is_8_connected_with_endpoints(p1, p2):
    xs, ys = V.line_pixels(20, 20, p1, p2)
    assert len(xs) == max(abs(p2[0] - p1[0]), abs(p2[1] - p1[1])) + 1
    pts = set(zip(xs.tolist(), ys.tolist()))
    assert tuple(p1) in pts and tuple(p2) in pts
    d = np.abs(np.diff(np.stack([xs, ys]), axis=1))
    assert d.max() <= 1 and (d.sum(0) >= 1).all()


def test_clip_line():
    ok, a, b = V.clip_line(10, 10, (-10, 5), (20, 5))
    assert ok and a == (0, 5) and b == (9, 5)
    ok, _, _ = V.clip_line(10, 10, (-5, -5), (-1, 20))
    assert not ok
    xs, ys = V.line_pixels(10, 10, (-10, -10), (30, 30))
    assert (xs == ys).all() and xs.min() == 0 and xs.max() == 9


def test_rectangle_outline_and_fill():
    img = np.zeros((30, 40, 3), np.uint8)
    V.rectangle(img, (5, 6), (20, 15), (1, 2, 3), 1)
    m = (img == (1, 2, 3)).all(2)
    want = np.zeros_like(m)
    want[6, 5:21] = want[15, 5:21] = True
    want[6:16, 5] = want[6:16, 20] = True
    assert (m == want).all()
    img[:] = 0
    V.rectangle(img, (35, 25), (50, 40), (9, 9, 9), -1)  # clipped fill, corners given in any order
    m = (img == 9).all(2)
    assert m.sum() == 5 * 5 and m[25:30, 35:40].all()


def test_add_weighted_float32_rounding():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (7, 9, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (7, 9, 3), dtype=np.uint8)
    out = V.add_weighted(a, 0.3, b, 0.7, 0)
    ref = np.clip(np.rint(a.astype(np.float32) * np.float32(0.3) + b.astype(np.float32) * np.float32(0.7)), 0, 255)
    assert (out == ref.astype(np.uint8)).all()
    dst = b.copy()
    V.add_weighted(a, 0.3, dst, 0.7, 0, dst)
    assert (dst == out).all()


def test_arrowed_line_wings():
    img = np.zeros((60, 60, 3), np.uint8)
    V.arrowed_line(img, (10, 30), (50, 30), (255, 0, 255), 1, tipLength=0.25)
    m = (img == (255, 0, 255)).all(2)
    assert m[30, 10:51].all()
    # wings end at cvRound(50 + 10 cos(pi +- pi/4)), cvRound(30 + 10 sin(pi +- pi/4)) = (43, 23) / (43, 37)
    assert m[23, 43] and m[37, 43]


def test_put_text_draws_inside_its_box():
    img = np.zeros((80, 200, 3), np.uint8)
    (w, h), base = V.get_text_size("ID:7 TRACKING", V.FONT_HERSHEY_SIMPLEX, 0.4, 1)
    assert 20 < w < 200 and 5 <= h <= 15
    V.put_text(img, "ID:7 TRACKING", (10, 40), V.FONT_HERSHEY_SIMPLEX, 0.4, (255, 255, 255), 1)
    ys, xs = np.nonzero((img == 255).all(2))
    assert len(ys) > 20
    assert ys.max() <= 40 + base + 1 and ys.min() >= 40 - h - 3 and xs.min() >= 8
    assert V._ascii("✅ DETECTED") == "? DETECTED"


def _track(tid, bbox, status, tsu=0, traj=None, vel=(0.0, 0.0)):
    return {"track_id": tid, "bbox": np.array(bbox, np.float64), "confidence": 0.9, "status": status,
            "time_since_update": tsu, "trajectory": traj or [], "velocity": np.array(vel)}


def test_visualizer_status_colours_fill_and_legend():
    frame = np.full((480, 640, 3), 40, np.uint8)
    keep = frame.copy()
    vz = V.TrajectoryVisualizer()
    tracks = [_track("T001", [300, 60, 340, 90], "detected", traj=[(280, 150), (290, 155), (300, 160)],
                     vel=(2.0, 1.0)),
              _track("T002", [150, 200, 190, 230], "predicted", tsu=3)]
    out = vz.draw_tracks(frame, tracks, detections=[[300, 60, 340, 90, 0.8]],
                         frame_info={"frame_number": 1, "state_changes": 0})
    assert (frame == keep).all()  # input untouched (the reference draws on image.copy())
    assert vz.frame_counter == 1
    # detected: 1-pixel green outline
    assert (out[75, 300] == (0, 255, 0)).all() and (out[90, 320] == (0, 255, 0)).all()
    assert (out[68, 305] == 40).all()
    # predicted, frame_counter 1 -> flash colour (0,220,255), box interior = 0.3 fill + 0.7 frame
    inner = out[215, 170].astype(int)
    want = np.rint(np.float32(0.3) * np.array((0, 220, 255), np.float32) + np.float32(0.7) * np.float32(40))
    assert (inner == want).all()
    assert (out[230, 170] == (0, 220, 255)).all()
    # trail (yellow) between the trajectory points, velocity arrow (magenta) from the centre
    assert (out[155, 290] == (255, 255, 0)).all()
    assert ((out == (255, 0, 255)).all(2)).sum() > 5
    # legend: black box in the bottom-right corner with a white 2-px frame
    assert (out[460, 420] == (0, 0, 0)).all() and (out[470, 500] == 255).all()
    # flash cycle: frames 6..11 use the plain 'predicted' colour at thickness 1
    vz.frame_counter = 5
    out2 = vz.draw_tracks(frame, tracks[1:])
    assert (out2[230, 170] == (0, 165, 255)).all()


def test_load_source_kinds(tmp_path):
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (12, 16, 3), dtype=np.uint8)
    assert FR.load_source(a)[0][1] is not None and (FR.load_source(a)[0][1] == a).all()
    st = np.stack([a, a[::-1]])
    got = FR.load_source(st)
    assert len(got) == 2 and (got[1][1] == a[::-1]).all()
    grey = a[:, :, 0]
    assert (FR.load_source(grey)[0][1] == grey[:, :, None]).all()
    from PIL import Image

    pil = Image.fromarray(a[:, :, ::-1].copy())  # RGB image
    assert (FR.load_source(pil)[0][1] == a).all()  # -> BGR, loaders.py:537-547
    FR.imwrite(str(tmp_path / "b.png"), a)
    FR.imwrite(str(tmp_path / "a.png"), a[::-1])
    np.save(tmp_path / "c.npy", np.stack([a, a, a]))
    one = FR.load_source(str(tmp_path / "b.png"))
    assert len(one) == 1 and (one[0][1] == a).all()
    d = FR.load_source(str(tmp_path))
    assert [os.path.basename(p).split(":")[0] for p, _ in d] == ["a.png", "b.png", "c.npy", "c.npy", "c.npy"]
    assert (d[0][1] == a[::-1]).all()
    g = FR.load_source(str(tmp_path / "*.png"))
    assert len(g) == 2
    mixed = FR.load_source([a, str(tmp_path / "b.png")])
    assert len(mixed) == 2
    with pytest.raises(TypeError):
        FR.load_source(3.5)
    with pytest.raises(ValueError):
        FR.load_source(a.astype(np.float32))


def test_video_reader_writer(tmp_path):
    rng = np.random.default_rng(2)
    frames = rng.integers(0, 256, (5, 8, 10, 3), dtype=np.uint8)
    with FR.VideoWriter(str(tmp_path / "out.npy"), 25, (10, 8)) as w:
        for f in frames:
            w.write(f)
        w.write(np.zeros((4, 4, 3), np.uint8))  # wrong size: dropped like cv2.VideoWriter
    cap = FR.VideoReader(str(tmp_path / "out.npy"))
    assert cap.isOpened() and cap.get(FR.CAP_PROP_FRAME_COUNT) == 5
    assert cap.get(FR.CAP_PROP_FRAME_WIDTH) == 10 and cap.get(FR.CAP_PROP_FRAME_HEIGHT) == 8
    got = list(cap)
    assert len(got) == 5 and all((g == f).all() for g, f in zip(got, frames))
    assert cap.read() == (False, None)
    wd = FR.VideoWriter(str(tmp_path / "pngs"), 25)
    for f in frames[:3]:
        wd.write(f)
    wd.release()
    rd = FR.VideoReader(str(tmp_path / "pngs"))
    assert rd.get(FR.CAP_PROP_FRAME_COUNT) == 3 and (rd.read()[1] == frames[0]).all()
    with pytest.raises(NotImplementedError):
        FR.VideoReader(str(tmp_path / "x.mp4"))
    with pytest.raises(NotImplementedError):
        FR.VideoWriter(str(tmp_path / "x.mp4"))


def test_y4m_reader(tmp_path):
    h, w = 4, 6
    p = tmp_path / "v.y4m"
    y = np.arange(h * w, dtype=np.uint8).reshape(h, w) + 100
    u = np.full((h, w), 128, np.uint8)
    v = np.full((h, w), 128, np.uint8)
    u2 = np.full((h // 2, w // 2), 160, np.uint8)
    with open(p, "wb") as f:
        f.write(f"YUV4MPEG2 W{w} H{h} F30:1 C444\n".encode())
        for _ in range(2):
            f.write(b"FRAME\n" + y.tobytes() + u.tobytes() + v.tobytes())
    cap = FR.VideoReader(str(p))
    assert cap.get(FR.CAP_PROP_FRAME_COUNT) == 2 and cap.get(FR.CAP_PROP_FPS) == 30
    ok, fr = cap.read()
    assert ok and (fr == y[:, :, None]).all()  # neutral chroma -> grey = Y
    cap.release()
    p2 = tmp_path / "v420.y4m"
    with open(p2, "wb") as f:
        f.write(f"YUV4MPEG2 W{w} H{h} F25:1 C420jpeg\n".encode())
        f.write(b"FRAME\n" + y.tobytes() + u2.tobytes() + np.full((h // 2, w // 2), 128, np.uint8).tobytes())
    ok, fr = FR.VideoReader(str(p2)).read()
    # 4:2:0 = OpenCV's I420 path, BT.601 limited range: Y' = (Y - 16) * 1220542, U - 128 = 32:
    # B = (Y' + 2^19 + 32 * 2116026) >> 20, G = (Y' + 2^19 + 32 * -409993) >> 20, R = (Y' + 2^19) >> 20
    yy = (y.astype(np.int64) - 16) * 1220542 + (1 << 19)
    assert ok and (fr[:, :, 0] == np.clip((yy + 32 * 2116026) >> 20, 0, 255)).all()
    assert (fr[:, :, 1] == np.clip((yy - 32 * 409993) >> 20, 0, 255)).all()
    assert (fr[:, :, 2] == np.clip(yy >> 20, 0, 255)).all()
    assert int(fr[0, 0, 2]) == round((100 - 16) * 255 / 219)  # limited range: 84 -> 98 (rounded)


def test_yolo_frames_accepts_paths(tmp_path):
    P = pkg_module("predictor")
    a = np.zeros((8, 8, 3), np.uint8)
    FR.imwrite(str(tmp_path / "f.png"), a)
    items = P.YOLO._frames(str(tmp_path / "f.png"))
    assert items[0][0].endswith("f.png") and items[0][1].shape == (8, 8, 3)


def test_compat_visualizer_is_the_package_one():
    import sys

    compat = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "yolo---small-target-recognition---kalman-trajectory-prediction_amd", "compat")
    sys.path.insert(0, compat)
    try:
        m = importlib.import_module("kalman.trajectory_visualizer")
        assert m.TrajectoryVisualizer is V.TrajectoryVisualizer
    finally:
        sys.path.remove(compat)


def test_compat_camera_motion_compensation_modules_resolve():
    """The reference's camera_motion_compensation imports (package and its three modules) resolve
    to this package's device-backed classes."""
    import sys

    compat = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "yolo---small-target-recognition---kalman-trajectory-prediction_amd", "compat")
    sys.path.insert(0, compat)
    try:
        T = pkg_module("tracker")
        Mo = pkg_module("motion")
        pk = importlib.import_module("camera_motion_compensation")
        mr = importlib.import_module("camera_motion_compensation.motion_reset_kalman_tracker")
        mc = importlib.import_module("camera_motion_compensation.motion_compensated_multi_tracker")
        gm = importlib.import_module("camera_motion_compensation.global_motion_detector")
        assert mr.MotionResetKalmanTracker is T.MotionResetKalmanTracker is pk.MotionResetKalmanTracker
        assert mc.MotionCompensatedMultiTracker is T.MotionCompensatedMultiTracker
        assert gm.GlobalMotionDetector is Mo.GlobalMotionDetector is pk.GlobalMotionDetector
        assert issubclass(T.MotionResetKalmanTracker, T.AircraftKalmanTracker)
    finally:
        sys.path.remove(compat)


def test_load_source_names(tmp_path):
    a = np.zeros((4, 4, 3), np.uint8)
    FR.imwrite(str(tmp_path / "image_7.png"), a)
    got = FR.load_source([a, str(tmp_path / "image_7.png"), a])
    assert [p for p, _ in got] == ["image0.jpg", str(tmp_path / "image_7.png"), "image2.jpg"]
