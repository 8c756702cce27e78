"""The global camera-motion checker on the CPU: sanity of the OpenCV restatements in
oracle/gmd_ref.py (cv2 is absent, so these pin behaviour, not cv2's bits), the reference's
numpy post-processing, and the tracker-side global branch of oracle/cmc_ref.py."""
import numpy as np
import pytest

from cmc_sequences import jumpy_sequence
from gmd_helpers import _sample, camera_sequence, make_world
from oracle import gmd_ref as G
from oracle.cmc_ref import RefCMCMultiTracker


def _frame(gray):
    return np.repeat(np.clip(gray, 0, 255).astype(np.uint8)[..., None], 3, axis=2)


def test_gray_is_the_fixed_point_luma():
    rng = np.random.default_rng(0)
    f = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    g = G.bgr_to_gray(f).astype(np.float64)
    ref = 0.114 * f[..., 0] + 0.587 * f[..., 1] + 0.299 * f[..., 2]
    assert np.abs(g - ref).max() <= 0.51


def test_pyramid_levels_and_pyr_down():
    assert G.pyramid_levels(512, 640) == 3
    assert G.pyramid_levels(100, 100) == 2  # 50, 25, then 13 <= 21 stops
    assert G.pyramid_levels(40, 40) == 0
    c = np.full((33, 47), 77, np.uint8)
    d = G.pyr_down(c)
    assert d.shape == (17, 24) and (d == 77).all()


def test_good_features_properties():
    g = G.bgr_to_gray(_frame(make_world(3, 256, 320)))
    corners, info = G.good_features(g, return_info=True)
    assert corners is not None and len(corners) == 200 and info["n_candidates"] > 200
    p = corners.reshape(-1, 2)
    d2 = ((p[:, None, :] - p[None, :, :]) ** 2).sum(-1)
    np.fill_diagonal(d2, 1e9)
    assert d2.min() >= 225  # minDistance 15
    e = info["eig"][p[:, 1].astype(int), p[:, 0].astype(int)]
    assert (np.diff(e) <= 0).all()  # strongest first
    assert G.good_features(np.full((64, 64), 9, np.uint8)) is None


@pytest.mark.parametrize("shift", [(0.0, 0.0), (2.5, -7.25), (-1.0, 13.0), (3.0, 31.0)])
def test_lk_recovers_a_translation(shift):
    world = make_world(5, 400, 480)
    h, w = 256, 320
    a = G.bgr_to_gray(_frame(_sample(world, 60, 60, h, w)))
    b = G.bgr_to_gray(_frame(_sample(world, 60 + shift[0], 60 + shift[1], h, w)))
    corners = G.good_features(a)
    nxt, status = G.optical_flow(a, b, corners)
    mv = (nxt - corners.reshape(-1, 2))[status == 1]
    assert status.mean() > 0.8
    med = np.median(mv, axis=0)
    assert np.allclose(med, [-shift[1], -shift[0]], atol=0.15), med


def test_detector_follows_the_camera():
    frames, off = camera_sequence(0, 30, whip_at=(20,))
    det = G.RefGlobalMotionDetector()
    n_est = 0
    for f in range(30):
        is_motion, mag, vec, reset = det.detect_motion(frames[f])
        if f == 0:
            assert (is_motion, mag, reset) == (False, 0.0, False)
            continue
        step = off[f] - off[f - 1]
        if isinstance(mag, np.float32) and np.hypot(*step) < 10:
            n_est += 1
            assert np.allclose(vec, [-step[1], -step[0]], atol=0.6), (f, vec, step)
    s = det.stats
    assert n_est >= 12 and s["total_detections"] == 29
    assert s["motion_events"] >= 5 and s["reset_triggers"] >= 2  # the fast pans and the whip


class Scripted:
    """A motion detector replaying scripted detect_motion results."""

    def __init__(self, results):
        self.results = list(results)

    def detect_motion(self, frame):
        return self.results.pop(0)


def scripted_results(T, seed=0):
    """Per-frame (is_motion, magnitude, vector, should_reset) covering the reset rules: large
    magnitudes, runs of moderate ones (mean of the last three > 30), unstable detection counts."""
    rng = np.random.default_rng(seed)
    out = [(False, 0.0, np.array([0.0, 0.0]), False)]
    for t in range(1, T):
        u = rng.random()
        if u < 0.55:
            out.append((False, 0.0, np.array([0.0, 0.0]), False))
            continue
        mag = np.float32(rng.choice([rng.uniform(0, 29), rng.uniform(30, 49), rng.uniform(50, 59),
                                     rng.uniform(60, 90)]))
        vec = np.array([mag, 0.0], np.float32)
        out.append((mag > 30.0, mag, vec, bool(mag > 50.0 or rng.random() < 0.3)))
    return out


def test_oracle_global_branch():
    T = 80
    seq = jumpy_sequence(3, K=10, T=T)
    res = scripted_results(T)
    ref = RefCMCMultiTracker(150, 1, 0.1, motion_detector=Scripted(res))
    resets = 0
    for t in range(T):
        before = ref.next_num
        out = ref.update(seq[t], frame=object())
        if ref.stats["global_resets"] > resets:
            resets = ref.stats["global_resets"]
            # every tracker is new, one per detection, ids continue from the counter
            assert [r["track_id"] for r in out] == list(range(before, before + len(seq[t])))
            assert all(r["age"] == 0 for r in out)
    assert ref.stats["global_motion_events"] == sum(bool(r[3]) for r in res)
    assert 3 <= ref.stats["global_resets"] < ref.stats["global_motion_events"]
