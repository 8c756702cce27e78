"""The HIP path against the committed golden fixtures (tests/golden/*.npz): the tracker kernel
(enhanced and motion-reset policies, config-3 / config-5 loads, reference defaults), the fp32
detector (YOLOv8n+P2 predict) and the device LetterBox resize.  Bars: decisions / ints exact,
tracker floats 1e-9, detector boxes 1e-4 (BASELINE north_star)."""
import hashlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import pkg

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402

pytestmark = pytest.mark.gpu


def _check_frames(outs, want):
    for t, frame in enumerate(outs):
        a, b = want["off"][t], want["off"][t + 1]
        wi, wf = want["ints"][a:b], want["flts"][a:b]
        assert len(frame) == b - a, f"frame {t}: {len(frame)} tracks vs {b - a}"
        gi = np.asarray([[int(d["track_id"][1:]), 0 if d["status"] == "detected" else 1, d["age"], d["hits"],
                          d["hit_streak"], d["time_since_update"], d.get("reset_count", 0)] for d in frame],
                        np.int32).reshape(-1, 7)
        gf = np.asarray([[*d["bbox"], d["confidence"]] for d in frame], np.float64).reshape(-1, 5)
        np.testing.assert_array_equal(gi, wi, err_msg=f"frame {t}")
        np.testing.assert_allclose(gf, wf, rtol=1e-9, atol=1e-9, err_msg=f"frame {t}")


@pytest.mark.parametrize("name", ["tracker_c3", "tracker_c5", "tracker_defaults"])
def test_tracker_kernel_matches_golden(name):
    yk = pkg()
    frames, args = G.tracker_inputs(name)
    trk = yk.EnhancedMultiTargetTracker(*args, max_tracks=2048, max_dets=512)
    outs = [trk.update(d) for d in frames]
    _check_frames(outs, G.load(name))
    want = G.load(name)["stats"][-1]
    s = trk.stats
    assert [s[k] for k in ("total_tracks_created", "total_tracks_terminated", "current_active_tracks",
                           "long_term_predictions", "successful_recoveries")] == want.tolist()


def test_motion_reset_tracker_matches_golden():
    yk = pkg()
    frames, args = G.cmc_inputs()
    trk = yk.MotionCompensatedMultiTracker(*args)
    outs = [trk.update(d) for d in frames]
    _check_frames(outs, G.load("cmc_jumpy"))


def test_fp32_detector_matches_golden():
    yk = pkg()
    P, ar, sd, frames = G.detector_setup()
    want = G.load("detector_n")
    yolo = yk.YOLO("yolov8-small.yaml", weights=sd, dtype="fp32", max_batch=2)
    res = yolo(frames)
    got = np.concatenate([r.boxes.data.cpu().numpy() for r in res])
    assert [len(r.boxes.data) for r in res] == want["n"].tolist()
    np.testing.assert_allclose(got[:, :4], want["dets"][:, :4], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(got[:, 4:], want["dets"][:, 4:], rtol=1e-4, atol=1e-6)


def test_device_letterbox_matches_golden():
    import importlib

    P = pkg()
    M = importlib.import_module(P.__name__ + ".model")
    want = G.load("letterbox")
    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    for (h, w), f in G.letterbox_inputs().items():
        dm = M.DeviceModel(M.Program(ar, sd, h, w, 640, 1, "fp32"))
        dm.detect(torch.from_numpy(f[None]).cuda(), 0.25, 0.7, 300)
        c = dm.letterboxed(1)[0]
        assert list(c.shape) == want[f"shape_{w}x{h}"].tolist()
        assert hashlib.sha256(c.tobytes()).digest() == want[f"sha_{w}x{h}"].tobytes()


def _f32bits(x):
    return np.asarray(x, np.float32).view(np.int32)


def test_global_motion_kernels_match_golden():
    """gmd.hip on the gmd_pan fixture: per-frame results bit-exact (float32 magnitude / vector),
    corners, LK status and the end points of tracked corners bit-exact, stats exact."""
    import importlib

    M = importlib.import_module(pkg().__name__ + ".motion")
    want = G.load("gmd_pan")
    frames = G.gmd_inputs()
    det = M.BatchedMotionDetector(1, frames.shape[1], frames.shape[2])
    for t, f in enumerate(frames):
        det.detect_host([f])
        m, st = det.download()
        r = want["res"][t]
        assert bool(m[0]["is_motion"]) == bool(r[0]) and bool(m[0]["should_reset"]) == bool(r[4]), f"frame {t}"
        if int(m[0]["magnitude_kind"]) == 1:
            assert _f32bits(m[0]["magnitude"]) == _f32bits(r[1]), f"frame {t}"
            assert (_f32bits(m[0]["vector"]) == _f32bits(r[2:4])).all(), f"frame {t}"
        else:
            assert r[1] == 0.0, f"frame {t}"
        if t:
            c, nx, sts = det.points(0)
            k = int(want["ncorners"][t])
            assert len(c) == k and (c == want["corners"][t, :k]).all(), f"frame {t}: corners"
            if k:
                assert (sts == want["status"][t, :k]).all(), f"frame {t}: status"
                ok = sts == 1
                assert (_f32bits(nx[ok]) == _f32bits(want["next"][t, :k][ok])).all(), f"frame {t}: LK end points"
    np.testing.assert_array_equal([int(st[0]["total_detections"]), int(st[0]["motion_events"]),
                                   int(st[0]["reset_triggers"])], want["stats"])


@pytest.mark.parametrize("tag", ["", "_scipy"], ids=["lap", "scipy"])
@pytest.mark.parametrize("kind", ["bytetrack", "botsort"])
def test_bytetrack_kernel_matches_golden(kind, tag):
    """bytetrack.hip on the bytetrack fixture: every frame's rows in order, ids / score / cls / idx
    exact, boxes within 1e-3 px (the ByteTrack parity bar)."""
    import importlib

    from oracle import bytetrack_ref as R

    BT = importlib.import_module(pkg().__name__ + ".bytetrack")
    want = G.load("bytetrack")
    rows, off = want[f"{kind}{tag}_rows"], want[f"{kind}{tag}_off"]
    cfg = dict(R.BOTSORT_CFG if kind == "botsort" else R.BYTETRACK_CFG)
    dev = BT.BatchedTracker(cfg, n_streams=1, max_tracks=256, max_dets=128, use_lap=tag == "")
    for t, (x, c, k) in enumerate(G.bytetrack_inputs()):
        dev.step([np.c_[x, c, k]])
        got = dev.download()[0]
        exp = rows[off[t]:off[t + 1]]
        assert got.shape == exp.shape, f"frame {t + 1}: {got.shape} vs {exp.shape}"
        if len(exp):
            np.testing.assert_array_equal(got[:, 4:8], exp[:, 4:8], err_msg=f"frame {t + 1}")
            np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-6, atol=1e-3, err_msg=f"frame {t + 1}")
