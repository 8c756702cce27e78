"""GPU parity: the HIP tracker (libyk.so, csrc/tracker.hip) against the numpy oracle
(oracle/tracker_ref.py) on seeded synthetic sequences.

Bar (BASELINE.json north_star): track-ID / association decisions identical, box and
Kalman-state floats within 1e-4 relative.  The test asserts a much tighter 1e-9: every
value is computed with the reference's exact float32/float64 operation order, the only
non-bitwise source being the device arctan2 (last-ulp; feeds direction/stability only).
The oracle runs with stable tie-breaking (the kernel's documented rule)."""
import numpy as np
import pytest

from conftest import pkg
from oracle.tracker_ref import RefMultiTracker, RefTrack

pytestmark = pytest.mark.gpu

INT_KEYS = ("track_id", "status", "age", "hits", "hit_streak", "time_since_update", "lost_frames", "is_lost",
            "is_stable_motion")
FLOAT_KEYS = ("confidence", "motion_confidence", "speed", "direction")
RTOL = 1e-9


def _close(a, b, what):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, what
    assert np.allclose(a, b, rtol=RTOL, atol=1e-9), f"{what}: {a} vs {b}"


def compare_frame(ours, ref, where):
    assert [o["track_id"] for o in ours] == [r["track_id"] for r in ref], where
    for o, r in zip(ours, ref):
        for k in INT_KEYS:
            assert o[k] == r[k], f"{where} {o['track_id']} {k}: {o[k]} vs {r[k]}"
        for k in FLOAT_KEYS:
            _close(o[k], r[k], f"{where} {o['track_id']} {k}")
        _close(o["bbox"], r["bbox"], f"{where} {o['track_id']} bbox")
        _close(o["velocity"], r["velocity"], f"{where} {o['track_id']} velocity")
        _close(np.array(o["trajectory"]).reshape(-1, 2), np.array(r["trajectory"], dtype=np.float64).reshape(-1, 2),
               f"{where} {o['track_id']} trajectory")


def run_pair(det_frames, max_lost=150, min_hits=1, thr=0.1):
    yk = pkg()
    ours = yk.EnhancedMultiTargetTracker(max_lost, min_hits, thr)
    ref = RefMultiTracker(max_lost, min_hits, thr, stable_ties=True)
    exact = total = 0
    for t, dets in enumerate(det_frames):
        a = ours.update(dets)
        b = ref.update(dets)
        compare_frame(a, b, f"frame {t}")
        for o, r in zip(a, b):
            total += 1
            exact += bool(np.array_equal(o["bbox"], r["bbox"]))
    assert ours.stats == ref.stats
    assert ours.frame_count == ref.frame_count and ours.next_track_id == ref.next_track_id
    return ours, ref, exact, total


@pytest.mark.parametrize("seed,K", [(0, 16), (1, 64)])
def test_tracker_matches_oracle_gt_sequences(seed, K):
    yk = pkg()
    sc = yk.synth.Scene(seed=seed, n_targets=K, n_frames=180)
    frames = [sc.detections(t) for t in range(sc.T)]
    ours, ref, exact, total = run_pair(frames)
    assert total > 0
    # boxes are computed with the reference's own rounding sequence: bitwise in practice
    assert exact / total > 0.99


def test_tracker_reference_defaults_and_float64_detections():
    yk = pkg()
    sc = yk.synth.Scene(seed=3, n_targets=12, n_frames=80)
    frames = [[[float(v) for v in d] for d in sc.detections(t)] for t in range(sc.T)]  # python floats
    run_pair(frames, max_lost=450, min_hits=3, thr=0.3)


def test_tracker_deletion_boundary_and_empty_frames():
    f = np.float32
    det = [[f(100), f(100), f(110), f(108), f(0.9)]]
    frames = [det, [[f(101), f(100), f(111), f(108), f(0.9)]]] + [[] for _ in range(160)] + [det]
    ours, ref, _, _ = run_pair(frames)
    assert ours.stats["total_tracks_terminated"] == 1


def test_tracker_exact_ties_stable_order():
    f = np.float32
    # two identical detections over one track: exact IoU tie, lowest detection index wins
    frames = [[[f(50), f(50), f(60), f(60), f(.9)]],
              [[f(50), f(50), f(60), f(60), f(.9)], [f(50), f(50), f(60), f(60), f(.8)]]] * 3
    run_pair(frames, thr=0.1)


def test_tracker_many_tracks_and_streams():
    yk = pkg()
    S = 4
    scenes = [yk.synth.Scene(seed=10 + s, n_targets=48 + 8 * s, n_frames=60) for s in range(S)]
    ms = yk.MultiStreamTracker(S, 150, 1, 0.1, max_tracks=256, max_dets=128)
    refs = [RefMultiTracker(150, 1, 0.1, stable_ties=True) for _ in range(S)]
    for t in range(60):
        per = [sc.detections(t) for sc in scenes]
        ms.step_host(per)
        rows, counts, stats = ms.download()
        for s in range(S):
            rb = refs[s].update(per[s])
            ours = [yk.tracker._row_to_dict(r, yk.tracker.track_id_of(r["track_num"])) for r in rows[s, : counts[s]]]
            compare_frame(ours, rb, f"stream {s} frame {t}")
            assert int(stats[s]["total_tracks_created"]) == refs[s].stats["total_tracks_created"]


@pytest.mark.parametrize("targets", [60, 100])
def test_tracker_every_pair_candidates_beyond_lds(targets):
    """iou_threshold 0 makes every (detection, track) pair a candidate.  At 2048 tracks x 512
    detections the walk's LDS area holds assoc_lds_cand = (163,840 - 133,632) / 12 = 2,517 of them
    (reported by the kernel, phase word 23): 60 targets (~3.6k pairs) take the LDS head + global
    tail path with the rounds on the dead box area (which holds (T*32 + D*32) / 12 = 6,826), 100
    targets (~10k) the rounds on global memory.  The candidate count is the kernel's own (phase
    word 12, counted on the pre-step tracks)."""
    yk = pkg()
    sc = yk.synth.Scene(seed=20 + targets, n_targets=targets, n_frames=12)
    T, Dm = 2048, 512
    ms = yk.MultiStreamTracker(1, 150, 1, 0.0, max_tracks=T, max_dets=Dm)
    ref = RefMultiTracker(150, 1, 0.0, stable_ties=True)
    most, cap = 0, None
    for t in range(12):
        dets = sc.detections(t)
        ms.step_host([dets])
        rows, counts, stats = ms.download()
        ph = ms.phase_us(0)
        if ph["n_cand"]:
            most = max(most, ph["n_cand"])
            cap = ph["lds_cand_cap"]
        rb = ref.update(dets)
        ours = [yk.tracker._row_to_dict(r, yk.tracker.track_id_of(r["track_num"])) for r in rows[0, : counts[0]]]
        compare_frame(ours, rb, f"frame {t}")
        assert int(stats[0]["overflow"]) == 0
    assert cap == 2517, cap
    dead_box_cap = (T * 32 + Dm * 32) // 12
    if targets == 60:
        assert cap < most <= dead_box_cap, (most, cap)
    else:
        assert most > dead_box_cap, most


def test_standalone_track_object_ops():
    yk = pkg()
    f = np.float32
    b0 = [f(100), f(100), f(110), f(108)]
    ours = yk.AircraftKalmanTracker(b0, track_id="A", max_lost_frames=150)
    ref = RefTrack(b0, "A", 150)
    for t in range(40):
        _close(ours.predict(), ref.predict(), f"predict {t}")
        if t % 5 != 4:
            b = [f(100 + 1.5 * t), f(100 + 0.5 * t), f(110 + 1.5 * t), f(108 + 0.5 * t)]
            ours.update(b)
            ref.update(b)
        else:
            ours.mark_as_lost()
            ref.mark_as_lost()
        _close(ours.x, ref.x, f"x {t}")
        _close(ours.P, ref.P, f"P {t}")
        compare_frame([ours.get_track_info()], [ref.get_track_info()], f"info {t}")
    for k in (1, 2, 7, 40):
        a, ca = ours.enhanced_long_term_predict(k)
        b, cb = ref.long_term_predict(k)
        _close(a, b, f"long-term {k}")
        _close(ca, cb, f"long-term conf {k}")


def test_multi_tracker_views_and_statistics():
    yk = pkg()
    sc = yk.synth.Scene(seed=5, n_targets=8, n_frames=40)
    ours = yk.EnhancedMultiTargetTracker(150, 1, 0.1)
    ref = RefMultiTracker(150, 1, 0.1, stable_ties=True)
    for t in range(40):
        ours.update(sc.detections(t))
        ref.update(sc.detections(t))
    so, sr = ours.get_statistics(), ref.get_statistics()
    assert so["tracker_details"] == [{**d, "confidence": pytest.approx(d["confidence"], rel=RTOL)} for d in sr["tracker_details"]]
    assert [t.track_id for t in ours.trackers] == [t.track_id for t in ref.trackers]
    for a, b in zip(ours.trackers, ref.trackers):
        _close(a.x, b.x, "view x")
        _close(a.P, b.P, "view P")
        assert a.age == b.age and a.hits == b.hits


@pytest.mark.timeout(900)
def test_config5_tracker_leg_256_tracks_150_frame_bursts():
    """BASELINE config 5's tracker leg: 256 targets per stream at 1280x1024 with 150-frame
    predict-only occlusion bursts (GT-injected detections, option (ii)), two streams
    stepped by one launch, every frame against the oracle; exact-IoU tie frames are counted."""
    import json

    yk = pkg()
    S, F = 2, 330
    scenes = [yk.synth.Scene(seed=500 + s, n_targets=256, n_frames=F, width=1280, height=1024,
                             occlusion_lengths=(1, 30, 149, 150, 150, 150)) for s in range(S)]
    ms = yk.MultiStreamTracker(S, 150, 1, 0.1, max_tracks=2048, max_dets=512)
    refs = [RefMultiTracker(150, 1, 0.1, stable_ties=True, fast_iou=True) for _ in range(S)]
    live_max = 0
    for t in range(F):
        per = [sc.detections(t) for sc in scenes]
        ms.step_host(per)
        rows, counts, stats = ms.download()
        for s in range(S):
            rb = refs[s].update(per[s])
            ours = [yk.tracker._row_to_dict(r, yk.tracker.track_id_of(r["track_num"])) for r in rows[s, : counts[s]]]
            compare_frame(ours, rb, f"stream {s} frame {t}")
            live_max = max(live_max, len(refs[s].trackers))
    for s in range(S):
        for k in refs[s].stats:
            assert int(stats[s][k]) == refs[s].stats[k], (s, k)
        assert int(stats[s]["overflow"]) == 0
    assert min(len(r.trackers) for r in refs) >= 256
    assert sum(r.stats["total_tracks_terminated"] for r in refs) > 0
    print("CONFIG5_TRACKER_LEG", json.dumps({"streams": S, "frames": F, "live_max": live_max,
                                             "live_end": [len(r.trackers) for r in refs],
                                             "terminated": [r.stats["total_tracks_terminated"] for r in refs],
                                             "tie_frames": [r.tie_frames for r in refs]}))


@pytest.mark.parametrize("max_lost,min_hits,thr,frames_n", [(30, 1, 0.1, 220), (450, 3, 0.3, 110), (0, 1, 0.1, 40)])
def test_tracker_event_messages_match_oracle(capsys, max_lost, min_hits, thr, frames_n):
    """verbose=True: the device event log (yk_tracker_set_events / yk_tracker_events) replayed by
    tracker.event_lines prints exactly the reference's lines, frame by frame -- init (:40),
    recoveries (kf.py:271 + multi:79, greedy match order), losses (kf.py:313 + multi:89, list
    order), creations (multi:101), deletions (multi:109), and the 100-frame statistics block with
    its per-tracker lines (multi:272-287) -- against RefMultiTracker(verbose=True).  max_lost 0
    removes a track on the step it is lost (a loss and a deletion in one step)."""
    yk = pkg()
    sc = yk.synth.Scene(seed=11, n_targets=24, n_frames=frames_n)
    ours = yk.EnhancedMultiTargetTracker(max_lost, min_hits, thr, verbose=True)
    a0 = capsys.readouterr().out
    ref = RefMultiTracker(max_lost, min_hits, thr, verbose=True, stable_ties=True)
    b0 = capsys.readouterr().out
    assert a0 == b0 and a0.startswith("增强版多目标跟踪器初始化完成")
    kinds = {"recover": 0, "lost": 0, "create": 0, "delete": 0, "stats": 0}
    for t in range(sc.T):
        dets = sc.detections(t)
        ours.update(dets)
        a = capsys.readouterr().out
        ref.update(dets)
        b = capsys.readouterr().out
        assert a == b, f"frame {t}:\n--- device\n{a}\n--- oracle\n{b}"
        kinds["recover"] += b.count("切换回检测模式")
        kinds["lost"] += b.count("切换到预测模式")
        kinds["create"] += b.count("创建新跟踪器")
        kinds["delete"] += b.count("删除跟踪器")
        kinds["stats"] += b.count("=== 跟踪统计")
    print("EVENT_MESSAGES", max_lost, min_hits, thr, kinds)
    assert kinds["lost"] > 0 and kinds["create"] > 0
    if max_lost > 0:  # (max_lost 0 removes every lost track at once: nothing can be recovered)
        assert kinds["recover"] > 0
    if max_lost != 450:
        assert kinds["delete"] > 0
    if frames_n >= 100:
        assert kinds["stats"] >= 1


@pytest.mark.parametrize("max_tracks, offset", [(256, 0), (151, 0), (256, 8)])
def test_download_async_pushes_the_rows_download_returns(max_tracks, offset):
    """yk_tracker_download_async (the per-step output push of the host-frame loop): counts, stats and
    every live row equal yk_tracker_download's, with 16-byte row stores (even max_tracks, aligned
    buffer), the 8-byte path (odd max_tracks: every other stream's rows start 8 bytes off; a host
    buffer 8 bytes off), and rows_per_stream cutting streams short."""
    import torch

    P = pkg()
    L = P._lib
    S = 4
    trk = P.tracker.MultiStreamTracker(S, max_lost_frames=30, min_hits=1, iou_threshold=0.1, max_tracks=max_tracks,
                                       max_dets=256)
    rng = np.random.default_rng(max_tracks + offset)
    for f in range(2):
        dets = []
        for s in range(S):
            n = int(rng.integers(10, 30)) + 15 * s
            xy = rng.uniform(0, 600, (n, 2))
            dets.append(np.concatenate([xy, xy + rng.uniform(5, 20, (n, 2)), rng.uniform(0.2, 1, (n, 1))], 1))
        trk.step_host(dets)
    rows_ref, counts_ref, stats_ref = (x.copy() for x in trk.download())
    assert (counts_ref > 0).all() and int(stats_ref["overflow"].sum()) == 0
    nb = S * max_tracks * L.TRACK_OUT_DTYPE.itemsize
    for rows_per_stream in (None, 17):
        raw = torch.zeros(nb + 16, dtype=torch.uint8, pin_memory=True)
        rows = raw[offset:offset + nb]
        counts = torch.zeros(S, dtype=torch.int32, pin_memory=True)
        stats = torch.zeros(S * L.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
        trk.download_async(rows, counts, stats, rows_per_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(counts.numpy(), counts_ref)
        assert stats.numpy().tobytes() == stats_ref.tobytes()
        got = rows.numpy().view(L.TRACK_OUT_DTYPE).reshape(S, max_tracks)
        for s in range(S):
            n = int(counts_ref[s]) if rows_per_stream is None else min(int(counts_ref[s]), rows_per_stream)
            assert got[s, :n].tobytes() == rows_ref[s, :n].tobytes()
            assert not got[s, n:].tobytes().strip(b"\0")  # nothing past the live rows
