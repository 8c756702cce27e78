"""Device global camera-motion detector (csrc/gmd.hip via yk_gmd_*) and the tracker's global
branch (yk_tracker_step_motion) against oracle/gmd_ref.py and oracle/cmc_ref.py.

Bar: corners (positions and order), Lucas-Kanade end points and status, and every
detect_motion result -- flags, float32 magnitude and vector -- bit-identical to the restatement
frame by frame; the direction consistency within 1e-5 (numpy's float32 arctan2 is its SIMD
implementation, up to 3 ulp from the device's correctly-rounded one); stats identical.  The
tracker branch: rows, ids and the global_motion_events / global_resets counters identical to
MotionCompensatedMultiTracker.update(detections, frame)."""

import numpy as np
import pytest
import torch

from cmc_sequences import jumpy_sequence
from conftest import pkg
from gmd_helpers import camera_sequence
from oracle.cmc_ref import RefCMCMultiTracker
from oracle.gmd_ref import RefGlobalMotionDetector
from test_cmc_gpu import compare
from test_gmd_cpu import Scripted, scripted_results

pytestmark = pytest.mark.gpu


def _motion():
    import importlib

    return importlib.import_module(pkg().__name__ + ".motion")


def _bits(x):
    return np.asarray(x, np.float32).view(np.int32)


def check_result(m, ref, ref_det, where):
    is_motion, mag, vec, reset = ref
    kind = 1 if isinstance(mag, np.float32) else 0
    assert int(m["magnitude_kind"]) == kind, where
    assert bool(m["is_motion"]) == bool(is_motion) and bool(m["should_reset"]) == bool(reset), where
    if kind:
        assert _bits(m["magnitude"]) == _bits(mag), f"{where}: magnitude {m['magnitude']} vs {mag}"
        assert (_bits(m["vector"]) == _bits(vec)).all(), f"{where}: vector {m['vector']} vs {vec}"
        c = ref_det.last_debug.get("consistency")
        if c is not None:
            assert abs(float(m["consistency"]) - float(c)) < 1e-5, where


def check_points(det, s, ref_det, where):
    c, nx, st = det.points(s)
    rc = ref_det.last_debug.get("corners")
    if rc is None:
        assert len(c) == 0, where
        return
    rc = rc.reshape(-1, 2)
    assert len(c) == len(rc) and (c == rc).all(), f"{where}: corners differ"
    if ref_det.last_debug.get("status") is None:
        return
    assert (st == ref_det.last_debug["status"]).all(), f"{where}: LK status differs"
    ok = st == 1
    assert (_bits(nx[ok]) == _bits(ref_det.last_debug["next"][ok])).all(), f"{where}: LK end points differ"


def run(seqs, points=True):
    M = _motion()
    S = len(seqs)
    F, H, W = seqs[0].shape[:3]
    det = M.BatchedMotionDetector(S, H, W)
    refs = [RefGlobalMotionDetector() for _ in range(S)]
    n_motion = n_reset = 0
    for f in range(F):
        det.detect_host([seqs[s][f] for s in range(S)])
        m, st = det.download()
        for s in range(S):
            r = refs[s].detect_motion(seqs[s][f])
            where = f"frame {f} stream {s}"
            check_result(m[s], r, refs[s], where)
            if points and f > 0:
                check_points(det, s, refs[s], where)
            n_motion += bool(r[0])
            n_reset += bool(r[3])
    for s in range(S):
        assert M.stats_dict(st[s]) == refs[s].get_stats()
    return n_motion, n_reset


def test_single_stream_pan_matches_oracle():
    frames, _ = camera_sequence(0, 30, whip_at=(20,))
    n_motion, n_reset = run([frames])
    assert n_motion >= 5 and n_reset >= 2


def test_batched_streams_match_oracle():
    seqs = [camera_sequence(10 + s, 18, whip_at=(7 + s,))[0] for s in range(3)]
    run(seqs)


def test_full_size_640x512():
    frames, _ = camera_sequence(4, 8, h=512, w=640, whip_at=(5,))
    run([frames])


def test_odd_frame_size():
    frames, _ = camera_sequence(6, 8, h=251, w=333, whip_at=(4,))
    run([frames])


def test_flat_frames_and_few_corners():
    """No corners (flat image) and fewer than 20 corners take the no-estimate returns."""
    flat = np.full((6, 128, 160, 3), 90, np.uint8)
    sparse = flat.copy()
    for k in range(6):
        for j in range(5):  # five bright squares -> a handful of corners
            sparse[k, 20 + 18 * j:28 + 18 * j, 30 + k:38 + k] = 200
    run([flat, sparse])


def test_detector_facade_and_reset():
    M = _motion()
    frames, _ = camera_sequence(1, 10, whip_at=())
    det, ref = M.GlobalMotionDetector(), RefGlobalMotionDetector()
    for f in range(10):
        a, b = det.detect_motion(frames[f]), ref.detect_motion(frames[f])
        assert type(a[1]) is type(b[1]) and a[1] == b[1] and bool(a[3]) == bool(b[3])
    assert det.get_stats() == ref.get_stats()
    det.reset_stats()
    ref.reset_stats()
    assert det.get_stats() == ref.get_stats()
    det.global_motion_threshold = 0.5  # set_global_motion_sensitivity-style threshold change
    ref.global_motion_threshold = 0.5
    for f in range(3):
        a, b = det.detect_motion(frames[f]), ref.detect_motion(frames[f])
        assert bool(a[0]) == bool(b[0])
    with pytest.raises(NotImplementedError):
        M.GlobalMotionDetector("feature_matching")


def _device_motion(records):
    t = torch.from_numpy(records.view(np.uint8).copy()).cuda()
    return t, t.data_ptr()


def test_tracker_global_branch_scripted():
    """yk_tracker_step_motion driven by scripted detect_motion results (every reset rule)."""
    yk = pkg()
    L = yk._lib
    S, T = 3, 90
    seqs = [jumpy_sequence(30 + s, K=10, T=T) for s in range(S)]
    scripts = [scripted_results(T, seed=s) for s in range(S)]
    ms = yk.MultiStreamTracker(S, 150, 1, 0.1, max_tracks=512, max_dets=64, policy=L.POLICY_MOTION_RESET)
    refs = [RefCMCMultiTracker(150, 1, 0.1, motion_detector=Scripted(scripts[s])) for s in range(S)]
    TR = yk.tracker
    for t in range(T):
        rec = np.zeros(S, L.MOTION_DTYPE)
        for s in range(S):
            is_motion, mag, vec, reset = scripts[s][t]
            rec[s] = (1, int(is_motion), int(reset), int(isinstance(mag, np.float32)), mag, vec, -1.0, 0, 0, 0, 0)
        keep, ptr = _device_motion(rec)
        per = [seqs[s][t] for s in range(S)]
        ms.step_host(per, motion=ptr)
        rows, counts, stats = ms.download()
        for s in range(S):
            rb = refs[s].update(per[s], frame=object())
            ours = [TR._reset_fields(r, TR._row_to_dict(r, TR.track_id_of(r["track_num"]))) for r in rows[s, : counts[s]]]
            compare(ours, rb, f"stream {s} frame {t}")
            assert int(stats[s]["global_motion_events"]) == refs[s].stats["global_motion_events"]
            assert int(stats[s]["global_resets"]) == refs[s].stats["global_resets"]
            assert int(stats[s]["individual_resets"]) == refs[s].stats["individual_resets"]
            assert int(stats[s]["tracking_recoveries"]) == refs[s].stats["tracking_recoveries"]
    assert sum(r.stats["global_resets"] for r in refs) >= 6


def test_motion_compensated_tracker_with_frames():
    """MotionCompensatedMultiTracker.update(detections, frame) end to end: device motion
    detector + tracker against the oracle's detector + tracker."""
    yk = pkg()
    T = 30
    frames, _ = camera_sequence(0, T, whip_at=(20,))
    dets = jumpy_sequence(5, K=8, T=T)
    ours = yk.tracker.MotionCompensatedMultiTracker(150, 1, 0.1)
    ref = RefCMCMultiTracker(150, 1, 0.1)
    for t in range(T):
        a = ours.update(dets[t], frames[t])
        b = ref.update(dets[t], frames[t])
        compare(a, b, f"frame {t}")
        assert bool(ours.frame_motion_info["should_reset"]) == bool(ref.frame_motion_info["should_reset"])
        assert all(o["global_motion"] is ours.frame_motion_info for o in a)
    assert ours.stats == ref.stats
    assert ref.stats["global_resets"] >= 1
    cs = ours.get_comprehensive_stats()
    assert cs["motion_detection"] == ref.motion_detector.get_stats()
    assert np.float64(cs["motion_history_avg"]) == np.float64(np.mean(ref.global_motion_history))


def test_many_candidates_take_the_windowed_selection():
    """Pixel noise has tens of thousands of local maxima: many LDS sort windows (2048 keys each,
    more than 16384 candidates), so the radix-select windows of select_kernel are exercised."""
    from oracle import gmd_ref as G

    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, (520, 660), dtype=np.uint8)
    frames = np.stack([np.repeat(base[k:k + 512, k:k + 640, None], 3, axis=2) for k in range(3)])
    _, info = G.good_features(G.bgr_to_gray(frames[0]), return_info=True)
    assert info["n_candidates"] > 16384
    run([frames])


def test_window_mode_matches_per_call_and_oracle():
    """yk_gmd_detect_window (n consecutive steps as n x S independent frame pairs in one launch
    sequence, chunks of 8, the post-processing stepping each stream's state in order) gives the
    per-call records bit for bit and the oracle's results: windows of 1, 3, 8 and 11 steps (a
    chunked one), odd frame size included; the two layouts refuse each other until reset."""
    M = _motion()
    L = pkg()._lib
    for h, w, seed in ((512, 640, 21), (251, 333, 22)):
        S, F = 3, 23
        seqs = [camera_sequence(seed + s, F, h=h, w=w, whip_at=(6 + s, 15))[0] for s in range(S)]
        frames = torch.from_numpy(np.stack(seqs, 1)).cuda()  # [F, S, H, W, 3]
        rec = L.MOTION_DTYPE.itemsize * S
        single = M.BatchedMotionDetector(S, h, w)
        out1 = torch.zeros((F, rec), dtype=torch.uint8, device="cuda")
        for f in range(F):
            single.detect_device(frames[f], out=out1[f].data_ptr())
        win = M.BatchedMotionDetector(S, h, w)
        out2 = torch.zeros((F, rec), dtype=torch.uint8, device="cuda")
        t = 0
        for n in (1, 3, 8, 11):
            win.detect_window([frames[f] for f in range(t, t + n)], out=out2[t].data_ptr())
            t += n
        assert t == F
        torch.cuda.synchronize()
        a, b = out1.cpu().numpy(), out2.cpu().numpy()
        assert a.tobytes() == b.tobytes(), [f for f in range(F) if a[f].tobytes() != b[f].tobytes()]
        m1, st1 = single.download()
        m2, st2 = win.download()
        assert m1.tobytes() == m2.tobytes() and st1.tobytes() == st2.tobytes()
        refs = [RefGlobalMotionDetector() for _ in range(S)]
        recs = a.view(L.MOTION_DTYPE).reshape(F, S)
        for f in range(F):
            for s in range(S):
                check_result(recs[f, s], refs[s].detect_motion(seqs[s][f]), refs[s], f"window mode frame {f} stream {s}")
        with pytest.raises(L.YKError):
            win.detect_device(frames[0])
        with pytest.raises(L.YKError):
            single.detect_window([frames[0]])
        win.reset()
        win.detect_device(frames[0])  # a reset detector takes either layout
