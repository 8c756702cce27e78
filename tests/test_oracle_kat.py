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


def test_fast_iou_matrix_is_the_scalar_iou_bit_for_bit():
    """oracle.tracker_ref.ref_iou_matrix_f32dets (the vectorised test-harness IoU) equals the
    scalar restatement of enhanced_multi_target_tracker.py:200-232 element for element,
    including ties between a det and a track coordinate, touching / disjoint boxes and
    degenerate (zero-area) boxes."""
    from oracle.tracker_ref import ref_iou_matrix_f32dets

    rng = np.random.default_rng(11)
    for trial in range(20):
        D, T = int(rng.integers(1, 40)), int(rng.integers(1, 40))
        c = rng.uniform(0, 100, (D, 2))
        wh = rng.uniform(0, 20, (D, 2))
        dets = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32)
        tc = rng.uniform(0, 100, (T, 2))
        twh = rng.uniform(0, 20, (T, 2))
        boxes = np.concatenate([tc - twh / 2, tc + twh / 2], 1)
        # plant exact coordinate ties, touching edges and copies
        for k in range(min(D, T) // 2):
            j = int(rng.integers(0, 4))
            boxes[k, j] = float(dets[k, j])
        if D > 2 and T > 2:
            boxes[1] = dets[1].astype(np.float64)
            boxes[2, 0] = float(dets[2, 2])  # touching: ix2 == ix1
            dets[0, 2] = dets[0, 0]          # zero-width det
        dl = [[d[0], d[1], d[2], d[3], f32(0.5)] for d in dets]
        want = np.array([[ref_iou(d[:4], b) for b in boxes] for d in dl])
        got = ref_iou_matrix_f32dets(dl, boxes)
        assert got.dtype == np.float64
        assert np.array_equal(got, want), trial


def test_fast_iou_tracker_equals_loop_tracker():
    from synth_helpers import scene_dets

    a = RefMultiTracker(150, 1, 0.1, stable_ties=True)
    b = RefMultiTracker(150, 1, 0.1, stable_ties=True, fast_iou=True)
    for dets in scene_dets(seed=5, n_targets=40, n_frames=60):
        ra, rb = a.update(dets), b.update(dets)
        assert [x["track_id"] for x in ra] == [x["track_id"] for x in rb]
        for x, y in zip(ra, rb):
            assert np.array_equal(x["bbox"], y["bbox"]) and x["confidence"] == y["confidence"]
