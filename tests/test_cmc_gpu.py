"""GPU parity of the motion-reset tracker policy (YK_POLICY_MOTION_RESET in csrc/tracker.hip,
MotionCompensatedMultiTracker in tracker.py) against the numpy restatement oracle/cmc_ref.py
of camera_motion_compensation/{motion_compensated_multi_tracker,motion_reset_kalman_tracker}.py.

Bar: association, reset decisions, ids (creation order), statuses and counters identical; box,
state, trajectory and motion values within 1e-9 relative (the float32/float64 operation order
is the reference's; the device arctan2 is the only non-bitwise source); the reset log's
averages, which the device accumulates in float64, within 1e-6."""
import numpy as np
import pytest

from cmc_sequences import jumpy_sequence
from conftest import pkg
from oracle.cmc_ref import RefCMCMultiTracker

pytestmark = pytest.mark.gpu

INT_KEYS = ("status", "age", "hits", "hit_streak", "time_since_update", "lost_frames", "is_lost",
            "is_stable_motion", "reset_count", "frames_since_reset", "motion_consistency", "status_suffix")
FLOAT_KEYS = ("confidence", "motion_confidence", "speed", "direction")


def _close(a, b, what, rtol=1e-9):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, what
    assert np.allclose(a, b, rtol=rtol, atol=1e-9), f"{what}: {a} vs {b}"


def _reason_texts(reasons):
    fmt = {"position": "position_jump_{:.1f}px", "velocity": "velocity_change_{:.1f}px/f", "size": "size_change_{:.2f}"}
    return [fmt[k].format(v) for k, v in reasons]


def compare(ours, ref, where):
    assert [o["track_id"] for o in ours] == [f"T{r['track_id']:03d}" for r in ref], where
    for o, r in zip(ours, ref):
        w = f"{where} {o['track_id']}"
        for k in INT_KEYS:
            assert o[k] == r[k], f"{w} {k}: {o[k]} vs {r[k]}"
        for k in FLOAT_KEYS:
            _close(o[k], r[k], f"{w} {k}")
        _close(o["bbox"], r["bbox"], f"{w} bbox")
        _close(o["velocity"], r["velocity"], f"{w} velocity")
        _close(np.array(o["trajectory"]).reshape(-1, 2), np.array(r["trajectory"], dtype=np.float64).reshape(-1, 2),
               f"{w} trajectory")
        a, b = o["reset_statistics"], r["reset_statistics"]
        assert a["total_resets"] == b["total_resets"], w
        if b["total_resets"]:
            assert a["reason_distribution"] == b["reason_distribution"], w
            _close(a["avg_confidence"], b["avg_confidence"], f"{w} avg_confidence", rtol=1e-6)
            _close(a["avg_motion_consistency"], b["avg_motion_consistency"], f"{w} avg_cons", rtol=1e-6)
            assert len(a["details"]) == len(b["details"]), w
            for da, db in zip(a["details"], b["details"]):
                assert da["frame"] == db["frame"], w
                assert da["reasons"] == _reason_texts(db["reasons"]), w
                _close(da["confidence"], db["confidence"], f"{w} detail confidence")
                _close(da["motion_consistency"], db["motion_consistency"], f"{w} detail consistency")


def run_pair(frames, max_lost=150, min_hits=1, thr=0.1):
    yk = pkg()
    ours = yk.tracker.MotionCompensatedMultiTracker(max_lost, min_hits, thr)
    ref = RefCMCMultiTracker(max_lost, min_hits, thr)
    for t, dets in enumerate(frames):
        compare(ours.update(dets), ref.update(dets), f"frame {t}")
    assert ours.stats == ref.stats
    return ours, ref


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_motion_reset_matches_oracle(seed):
    ours, ref = run_pair(jumpy_sequence(seed))
    assert ref.stats["individual_resets"] > 5  # the sequence exercises the reset path


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_motion_reset_cluttered_detections(seed):
    """Two overlapping boxes for most targets (the planted detector's clutter): the association
    rounds run long chains, and a pair whose detection and track were both matched in earlier
    rounds -- detection 0 with the track at list position 0 among them -- stays a candidate while
    later rounds still run (the reversed-rank round bookkeeping must not re-match it)."""
    # seed 1 (101): three frames where the old bookkeeping re-matched pair (0, 0) (checked on the
    # CPU by simulating the rounds against cmc_greedy)
    run_pair(jumpy_sequence(100 + seed, K=12, T=90, dup=1.0, shuffle=False))


def test_motion_reset_float64_detections_and_deletions():
    frames = [[[float(v) for v in d] for d in f] for f in jumpy_sequence(7, K=8, T=120)]
    run_pair(frames, max_lost=20)


def test_motion_reset_multi_stream_batch():
    """Four streams stepped by one kernel launch, each against its own oracle."""
    yk = pkg()
    S = 4
    seqs = [jumpy_sequence(20 + s, K=10, T=90) for s in range(S)]
    ms = yk.MultiStreamTracker(S, 150, 1, 0.1, max_tracks=512, max_dets=64, policy=yk._lib.POLICY_MOTION_RESET)
    refs = [RefCMCMultiTracker(150, 1, 0.1) for _ in range(S)]
    T = yk.tracker
    for t in range(90):
        per = [seqs[s][t] for s in range(S)]
        ms.step_host(per)
        rows, counts, stats = ms.download()
        for s in range(S):
            rb = refs[s].update(per[s])
            ours = [T._reset_fields(r, T._row_to_dict(r, T.track_id_of(r["track_num"]))) for r in rows[s, : counts[s]]]
            compare(ours, rb, f"stream {s} frame {t}")
            assert int(stats[s]["individual_resets"]) == refs[s].stats["individual_resets"]


def test_motion_reset_exact_tie_takes_highest_detection():
    """Two detections with exactly equal IoU against one track (mirror images about its
    centre): the (iou, d, t)-descending order gives the track to the LATER detection (the
    enhanced tracker's stable order gives it to the first)."""
    f = np.float32
    t0 = [f(50), f(50), f(60), f(60), f(.9)]
    d0 = [f(49), f(50), f(59), f(60), f(.9)]
    d1 = [f(51), f(50), f(61), f(60), f(.8)]
    ours, ref = run_pair([[t0], [d0, d1], [d0, d1]])
    assert ref.trackers[0].x[0] > 55.0  # track 1 moved toward d1


def test_standalone_motion_reset_track_object():
    """camera_motion_compensation.MotionResetKalmanTracker as one object (the compat module):
    predict / update / mark_as_lost / get_track_info / get_reset_statistics and the reset
    attributes, on a box path with position jumps, a size change, a velocity change and missed
    frames, against oracle/cmc_ref.RefResetTrack step by step."""
    import os
    import sys

    from conftest import REPO
    from oracle.cmc_ref import RefResetTrack

    sys.path.insert(0, os.path.join(REPO, pkg().__name__, "compat"))
    try:
        from camera_motion_compensation.motion_reset_kalman_tracker import MotionResetKalmanTracker
    finally:
        sys.path.pop(0)
    f = np.float32
    path = []
    x, y, w, h = 100.0, 120.0, 12.0, 9.0
    for t in range(60):
        if t in (12, 31):
            x += 55.0  # position jump > 40 px
        if t == 22:
            w, h = w * 1.6, h * 1.6  # size change > 0.3
        if 40 <= t < 44:
            x += 20.0 * (t - 39)  # accelerating: velocity change
        x, y = x + 1.5, y + 0.7
        path.append(None if t in (17, 18, 47) else [f(x - w / 2), f(y - h / 2), f(x + w / 2), f(y + h / 2)])
    b0 = [f(98.0), f(115.0), f(110.0), f(124.0)]
    ours = MotionResetKalmanTracker(b0, track_id="T001", max_lost_frames=150)
    ref = RefResetTrack(b0, "T001", 150)
    for t, box in enumerate(path):
        _close(ours.predict(), ref.predict(), f"frame {t} predict")
        if box is None:
            ours.mark_as_lost()
            ref.mark_as_lost()
        else:
            ours.update(box)
            ref.update(box)
        a, b = ours.get_track_info(), ref.get_track_info()
        for k in INT_KEYS:
            assert a[k] == b[k], f"frame {t} {k}: {a[k]} vs {b[k]}"
        _close(a["bbox"], b["bbox"], f"frame {t} bbox")
        assert ours.reset_count == ref.reset_count and ours.last_reset_frame == ref.last_reset_frame
        _close(ours.motion_consistency, ref.motion_consistency, f"frame {t} consistency")
    assert ref.reset_count >= 2, ref.reset_count  # the jumps at frames 12 and 31 (cooldown 15)
    sa, sb = ours.get_reset_statistics(), ref.get_reset_statistics()
    assert sa["total_resets"] == sb["total_resets"] and sa["reason_distribution"] == sb["reason_distribution"]
    _close(sa["avg_confidence"], sb["avg_confidence"], "avg_confidence", rtol=1e-6)
    assert [d["frame"] for d in sa["details"]] == [d["frame"] for d in sb["details"]]
