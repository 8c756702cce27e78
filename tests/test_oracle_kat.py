"""Pin the CPU oracle (oracle/tracker_ref.py) to the known-answer tests of SURVEY.md §8c.

The reference's Python cannot be run here (SURVEY §8c denial), and its own test-suite pins
no numbers on this path, so these KATs -- computed from the reference formulas -- are the
oracle's pins."""
import numpy as np
import pytest

from oracle.tracker_ref import RefMultiTracker, RefTrack, ref_greedy_assign, ref_iou

f32 = np.float32


def _track_kat():
    t = RefTrack([f32(100), f32(100), f32(110), f32(108)], "T001", 150)
    t.predict()
    return t


def test_kat_predict_covariance():
    t = _track_kat()
    assert np.array_equal(np.diag(t.P), [150.1, 150.1, 51.01, 51.01, 100.1, 100.1, 1.001, 1.001])
    assert t.P[0, 4] == 100.0


def test_kat_update_state_and_asymmetric_covariance():
    t = _track_kat()
    t.update([f32(102), f32(100), f32(112), f32(108)])
    assert t.x.tolist() == [106.87507807620237, 104.0, 10.0, 8.0, 1.249219237976265, 0.0, 0.0, 0.0]
    d = np.diag(t.P)
    assert d[0] == 9.375390381011865 and d[2] == 8.36092443861662
    assert d[4] == 37.63903810118674 and d[6] == 0.984609244386166
    assert t.P[0, 4] == 6.246096189881323 and t.P[4, 0] == 6.246096189881314
    assert np.count_nonzero(t.P) == 16


def test_kat_ten_more_predicts():
    t = _track_kat()
    t.update([f32(102), f32(100), f32(112), f32(108)])
    for _ in range(10):
        t.predict()
    assert t.x[0] == 119.367270455965
    assert t.P[0, 0] == 3927.7011242973122


def test_kat_iou():
    t = RefTrack([f32(100), f32(100), f32(110), f32(108)], "T001", 150)
    pb = t.predict()
    assert ref_iou([f32(102), f32(100), f32(112), f32(108)], pb) == 64 / 96


def test_kat_counters_quirk_a():
    """Created frame 1, matched frame 2, missed frames 3 and 4 (SURVEY §8c counter KAT)."""
    m = RefMultiTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
    m.update([[f32(100), f32(100), f32(110), f32(108), f32(0.9)]])
    m.update([[f32(101), f32(100), f32(111), f32(108), f32(0.9)]])
    out3 = m.update([])
    assert (out3[0]["age"], out3[0]["time_since_update"], out3[0]["status"], out3[0]["confidence"]) == (3, 2, "predicted", 1.0)
    trk = m.trackers[0]
    x_before = trk.x.copy()
    out4 = m.update([])
    o = out4[0]
    assert (o["age"], o["time_since_update"], o["status"]) == (4, 3, "predicted")
    assert o["confidence"] == 1 - 2 / 75
    # box = F^2 x computed without mutating the state (quirk B, low-confidence branch)
    s = trk.x.copy()
    for _ in range(2):
        s = trk.F @ s
    assert np.array_equal(o["bbox"], np.array([s[0] - s[2] / 2.0, s[1] - s[3] / 2.0, s[0] + s[2] / 2.0, s[1] + s[3] / 2.0]))
    assert not np.array_equal(trk.x, x_before)  # the regular predict of frame 4 did advance x


def test_kat_lifecycle_deleted_on_150th_miss():
    m = RefMultiTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
    m.update([[f32(100), f32(100), f32(110), f32(108), f32(0.9)]])
    misses = 0
    while m.trackers:
        m.update([])
        misses += 1
        assert misses <= 200
    assert misses == 150


def test_greedy_stable_tie_break_matches_sequential_scan():
    iou = np.array([[0.5, 0.5], [0.5, 0.2]])
    assert ref_greedy_assign(iou, 0.1, stable=True) == [(0, 0), (1, 1)]


@pytest.mark.parametrize("seed", range(3))
def test_inv_s_is_reciprocal_diagonal(seed):
    """inv(S) == diag(1/S_jj) bitwise: the HIP kernel relies on it (tracker.hip header)."""
    rng = np.random.default_rng(seed)
    for _ in range(200):
        s = rng.uniform(10.0, 5000.0, 4)
        assert np.array_equal(np.linalg.inv(np.diag(s)), np.diag(1.0 / s))


# ---------------------------------------------------------------- motion-reset variant
def _still_then_jump(dx, n_still=20):
    f = np.float32
    still = [[f(100), f(100), f(300), f(260), f(0.9)]]  # large box: a 50 px jump keeps IoU 0.6
    jumped = [[f(100 + dx), f(100), f(300 + dx), f(260), f(0.9)]]
    return [still] * n_still + [jumped]


def test_cmc_oracle_position_jump_resets():
    """A 50 px jump of a 200x160 box after 20 still frames (IoU 0.6, still matched): distance
    50 > 40 -> factor 1.25; the score history
    (nine ~0 scores and 1.25) has consistency 1 - var/(mean + 0.1) = 0.375 >= 0.3, so the
    confidence stays 1.25 > 1.0 and the filter resets to the new box with zero velocity."""
    from oracle.cmc_ref import RefCMCMultiTracker
    tr = RefCMCMultiTracker(150, 1, 0.1)
    for dets in _still_then_jump(50):
        out = tr.update(dets)
    t = tr.trackers[0]
    assert len(tr.trackers) == 1 and t.reset_count == 1 and tr.stats["individual_resets"] == 1
    assert [k for k, _ in t.reset_log[0]["reasons"]] == ["position"]
    assert abs(float(t.reset_log[0]["confidence"]) - 1.25) < 1e-3
    assert t.x[0] == np.float32(250.0) and np.all(t.x[4:] == 0)
    assert out[0]["frames_since_reset"] == 0 and out[0]["status_suffix"].startswith(" | ")


def test_cmc_oracle_small_jump_keeps_filter():
    from oracle.cmc_ref import RefCMCMultiTracker
    tr = RefCMCMultiTracker(150, 1, 0.1)
    for dets in _still_then_jump(8):
        tr.update(dets)
    assert tr.trackers[0].reset_count == 0


def test_cmc_greedy_tie_order():
    """(iou, d, t) tuples sorted in reverse: on an exact IoU tie the larger detection index
    wins the track (motion_compensated_multi_tracker.py:262-274)."""
    from oracle.cmc_ref import cmc_greedy
    iou = np.array([[0.5, 0.2], [0.5, 0.0]])
    assert cmc_greedy(iou, 0.1) == [(1, 0), (0, 1)]
    assert cmc_greedy(np.array([[0.1]]), 0.1) == []  # strict >
