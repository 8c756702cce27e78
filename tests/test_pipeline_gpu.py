"""End-to-end GPU parity: frames in HBM -> detector -> NMS -> tracker (device hand-off),
against the oracle chain (torch-CPU detector -> numpy tracker) per stream, plus the
reference driver's loop through the compat ``ultralytics`` / ``kalman`` packages."""
import importlib
import json
import os
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, pkg
from oracle import detector_ref as D
from oracle.tracker_ref import RefMultiTracker

pytestmark = pytest.mark.gpu


def _layers(ar):
    return [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
            for Ly in ar.layers]


def _trk_dicts(P, rows, n):
    return [P.tracker._row_to_dict(r, P.tracker.track_id_of(r["track_num"])) for r in rows[:n]]


def test_stream_pipeline_fp32_matches_oracle_chain():
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 2, 10
    pipe = pipeline.StreamPipeline("yolov8-small.yaml", S, (512, 640), "fp32", seed=0, max_tracks=256)
    ar = pipe.prog.ar
    ref = D.RefDetector(_layers(ar), pipe.prog.sd, P.arch.detect_strides(ar))
    scenes = [P.synth.Scene(seed=20 + s, n_targets=20, n_frames=F) for s in range(S)]
    refs = [RefMultiTracker(150, 1, 0.1, stable_ties=True) for _ in range(S)]
    torch.set_num_threads(8)
    for t in range(F):
        fr = [sc.frame(t) for sc in scenes]
        pipe.run(torch.from_numpy(np.stack(fr)).cuda())
        rows, counts, _ = pipe.tracker.download()
        want, _ = D.predict(ref, fr)
        for s in range(S):
            dets = [[b[0], b[1], b[2], b[3], b[4]] for b in want[s][:, :5].numpy()]
            rb = refs[s].update(dets)
            ours = _trk_dicts(P, rows[s], int(counts[s]))
            assert [o["track_id"] for o in ours] == [r["track_id"] for r in rb], (t, s)
            for o, r in zip(ours, rb):
                assert (o["status"], o["age"], o["hits"], o["time_since_update"]) == \
                    (r["status"], r["age"], r["hits"], r["time_since_update"])
                np.testing.assert_allclose(o["bbox"], r["bbox"], rtol=1e-4, atol=1e-3)
                np.testing.assert_allclose(o["confidence"], r["confidence"], rtol=1e-4)


# Scene seed of the strict driver-loop test.  The scene's tracks include many coasting
# duplicates, so some frames' greedy association is decided by IoU gaps far below the fp32
# detector's chain-to-chain IoU spread (~1e-6): seed 4's oracle chain has a 3.8e-8 gap (frame 89)
# and a 2.8e-7 one at frame 75 where two duplicate tracks swap (tools/driver_diag.py).  A strict
# chain test only measures parity on a scene whose oracle chain is decided by margins well above
# that spread; seed 8's smallest margin is 1.5e-5 (tools/driver_scene_margin.py), asserted below.
DRIVER_SEED = 8
DRIVER_MIN_MARGIN = 1e-5


def _driver_scene(P, n_frames, seed=DRIVER_SEED):
    """40 targets over n_frames with the lifecycle events the driver's statistics count: the
    scene's own occlusion bursts, plus targets forced out for 1-3 frames (lost -> recovered) and
    three forced out from frame 3 to the end (their tracks reach the 150-miss deletion unless a
    neighbouring detection keeps them alive; at least one is deleted)."""
    sc = P.synth.Scene(seed=seed, n_targets=40, n_frames=n_frames + 1)
    for k, (t0, L) in enumerate(((6, 1), (9, 2), (14, 3), (20, 2), (31, 1), (44, 3))):
        sc.visible[t0:t0 + L, k] = False
    sc.visible[3:, 37:40] = False
    return sc


def _run_driver(tmp_path, seed, F=160):
    """kalman/aircraft_detection_tracking.py:45-161 run unchanged through the compat imports --
    ``YOLO(model_path)`` with no dtype argument (so the drop-in default), frames read through the
    VideoCapture-like reader (a .npy frame stack, since no codec is in the image), the per-frame
    body of :88-131, the visualizer and the VideoWriter-like sink.  Returns what the chain check
    needs: the model, the frames and every frame's (float32 detections, track dicts)."""
    sys.path.insert(0, os.path.join(REPO, pkg().__name__, "compat"))
    try:
        from kalman.enhanced_multi_target_tracker import EnhancedMultiTargetTracker
        from kalman.trajectory_visualizer import TrajectoryVisualizer
        from ultralytics import YOLO
    finally:
        sys.path.pop(0)

    P = pkg()
    FR = P.frames
    sc = _driver_scene(P, F, seed)
    frames = np.stack([sc.frame(t) for t in range(F)])
    np.save(tmp_path / "seq.npy", frames)
    # --- the driver, as written (aircraft_detection_tracking.py:45-52, 58-161) ---------------------
    model = YOLO("yolov8s-small.yaml")
    assert model.dtype == "fp32"  # the drop-in default is the reference's arithmetic
    tracker = EnhancedMultiTargetTracker(max_lost_frames=150, min_hits=1, iou_threshold=0.1)
    vis = TrajectoryVisualizer()
    cap = FR.VideoReader(str(tmp_path / "seq.npy"))
    fps = int(cap.get(FR.CAP_PROP_FPS))
    width, height = int(cap.get(FR.CAP_PROP_FRAME_WIDTH)), int(cap.get(FR.CAP_PROP_FRAME_HEIGHT))
    out = FR.VideoWriter(str(tmp_path / "result.npy"), fps, (width, height))
    detection_frames = prediction_frames = state_changes = frame_count = 0
    last = {}
    per_frame = []
    while True:
        ret, frame = cap.read()
        if not ret:
            break
        frame_count += 1
        results = model(frame, verbose=False)
        detections = []
        if len(results) > 0 and results[0].boxes is not None:
            boxes = results[0].boxes.xyxy.cpu().numpy()
            scores = results[0].boxes.conf.cpu().numpy()
            for box, score in zip(boxes, scores):
                if score > 0.1:
                    detections.append([box[0], box[1], box[2], box[3], score])
        assert all(isinstance(v, np.float32) for d in detections for v in d)
        tracks = tracker.update(detections)
        per_frame.append((np.array(detections, np.float32).reshape(-1, 5), tracks))
        cur = {}
        for tr in tracks:
            cur[tr["track_id"]] = tr["status"]
            if tr["track_id"] in last and last[tr["track_id"]] != tr["status"]:
                state_changes += 1
            detection_frames += tr["status"] == "detected"
            prediction_frames += tr["status"] == "predicted"
        last = cur
        frame_info = {"frame_number": frame_count, "detections": len(detections), "tracks": len(tracks),
                      "detection_frames": detection_frames, "prediction_frames": prediction_frames,
                      "state_changes": state_changes}
        if frame_count <= 8 or frame_count % 40 == 0:  # drawing is host work; a sample suffices
            vis_frame = vis.draw_tracks(frame, tracks, detections, frame_info)
            assert vis_frame.shape == frame.shape and (vis_frame != frame).any()
            out.write(vis_frame)
    cap.release()
    out.release()
    assert frame_count == F and tracker.frame_count == F
    assert results[0].boxes.xyxy.is_cuda and results[0].orig_shape == (512, 640)
    assert detection_frames > 0 and prediction_frames > 0 and state_changes > 0
    return dict(model=model, frames=frames, per_frame=per_frame, tracker=tracker, state_changes=state_changes)


def _check_driver_chain(run, assoc_tie_margin=None):
    """The oracle chain on the driver's frames: per frame the detections equal the oracle's row for
    row (1e-4 relative, 1e-3 px; scores 1e-4); the track dicts equal the oracle chain's (oracle
    detector -> oracle RefMultiTracker(150, 1, 0.1)): decisions identical, boxes within 1e-4 of
    the box's scale; and on every frame they equal the oracle tracker fed the GPU's own detections
    (1e-9, test_tracker_gpu.compare_frame).

    assoc_tie_margin=None: strict, no allowance.  A number: the association near-tie policy (the
    NMS near-tie policy of tests/test_bench_pipeline_gpu.py applied to the tracker) -- a frame
    whose decisions differ from the oracle chain's is accepted only when that frame's oracle
    greedy association had a pick decided by less than assoc_tie_margin (gpu_helpers.assign_margin:
    the IoU gap to the free pair it beat, or to the gate); it is counted, both chains' IoUs of
    the differing tracks are printed, and the oracle chain is resynced to the GPU's pick (its
    tracker takes the state of the oracle tracker fed the GPU's detections, which equals the
    device tracker at 1e-9), so every later frame is still compared."""
    import copy

    from gpu_helpers import assign_margin, decisions, dets_match
    from test_tracker_gpu import compare_frame

    P = pkg()
    model, frames, per_frame = run["model"], run["frames"], run["per_frame"]
    F = len(per_frame)
    ref = D.RefDetector(_layers(model.arch), model.state_dict, P.arch.detect_strides(model.arch))
    trk = RefMultiTracker(150, 1, 0.1, stable_ties=True, fast_iou=True)
    iso = RefMultiTracker(150, 1, 0.1, stable_ties=True, fast_iou=True)
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    n_tracks, box_rel, margin, flips = 0, 0.0, np.inf, []
    for t in range(F):
        want, _ = D.predict(ref, [frames[t]])
        wd = want[0][:, :5].numpy()
        got_d, ours = per_frame[t]
        assert dets_match(got_d, wd) == "same", (f"frame {t}: detections differ from the oracle's", got_d, wd)
        rb = trk.update([[b[0], b[1], b[2], b[3], b[4]] for b in wd])
        fm = assign_margin(trk.last_iou, 0.1) if trk.last_iou is not None else np.inf
        margin = min(margin, fm)
        ri = iso.update([[b[0], b[1], b[2], b[3], b[4]] for b in got_d])
        compare_frame(ours, ri, f"isolated tracker frame {t}")
        if decisions(ours) != decisions(rb):
            assert assoc_tie_margin is not None and fm < assoc_tie_margin, \
                (f"frame {t}: association decisions differ (oracle margin {fm:.3g})", decisions(ours), decisions(rb))
            ids = {d[0] for d in set(decisions(ours)) ^ set(decisions(rb))}
            flips.append({"frame": t, "oracle_margin": fm, "tracks": sorted(str(i) for i in ids),
                          "oracle_iou_max": [float(trk.last_iou.max())], "gpu_chain_iou_max": [float(iso.last_iou.max())]})
            print("ASSOC_NEAR_TIE_FLIP", flips[-1])
            trk = copy.deepcopy(iso)  # resync: the oracle chain continues from the GPU's pick
            continue
        for o, r in zip(ours, rb):
            scale = float(np.max(np.abs(r["bbox"])))
            dev = float(np.max(np.abs(np.asarray(o["bbox"]) - r["bbox"])))
            assert dev <= 1e-4 * scale + 1e-3, (t, o["track_id"], o["bbox"], r["bbox"])
            box_rel = max(box_rel, dev / max(scale, 1.0))
            n_tracks += 1
    st = iso.stats
    assert st["total_tracks_terminated"] >= 1 and st["successful_recoveries"] > 0, st  # deletion + recovery ran
    assert run["tracker"].get_statistics()["total_tracks_terminated"] == st["total_tracks_terminated"]
    return dict(frames=F, chain_track_outputs_compared=n_tracks, max_box_rel_dev=box_rel, min_assign_margin=margin,
                assoc_near_tie_flips=flips, stats=dict(st), oracle_chain_stats=dict(trk.stats),
                state_changes=run["state_changes"])


@pytest.mark.timeout(900)
def test_reference_driver_loop_through_compat_packages(tmp_path):
    """The reference driver loop (see _run_driver) held to the oracle chain under the strict bar:
    no near-tie allowance at all, on a scene whose oracle chain is decided by association margins
    >= DRIVER_MIN_MARGIN (asserted).  160 frames so the 150-miss deletion happens inside the loop."""
    out = _check_driver_chain(_run_driver(tmp_path, DRIVER_SEED))
    F = out["frames"]
    assert out["chain_track_outputs_compared"] > 0
    assert out["min_assign_margin"] >= DRIVER_MIN_MARGIN, out["min_assign_margin"]  # well conditioned
    assert out["oracle_chain_stats"] == out["stats"]  # the oracle chain and the isolated oracle tracker agree
    print("DRIVER_LOOP", {k: v for k, v in out.items() if k != "assoc_near_tie_flips"}, F)


@pytest.mark.timeout(900)
def test_reference_driver_loop_ill_conditioned_scene_counted_ties(tmp_path):
    """The same driver loop on the rounds-2/3 scene (seed 4), whose many coasting duplicate tracks
    give association margins of 3.8e-8 (frame 89) and 2.8e-7 (frame 75) -- below the ~1e-6 IoU
    spread of two fp32 detector chains, so no implementation can be held to the oracle's pick there.
    Under the association near-tie policy (_check_driver_chain): every frame compared, a differing
    frame accepted only at an oracle margin < 1e-5, counted and resynced; at most 3 such frames."""
    out = _check_driver_chain(_run_driver(tmp_path, 4), assoc_tie_margin=1e-5)
    print("DRIVER_LOOP_SEED4", {k: v for k, v in out.items() if k != "assoc_near_tie_flips"},
          "flips", len(out["assoc_near_tie_flips"]))
    assert out["min_assign_margin"] < 1e-5  # the scene really is ill conditioned
    assert len(out["assoc_near_tie_flips"]) <= 3, out["assoc_near_tie_flips"]


def _plan_at_forward_batch(pipe, path="plans/s_640x512_i640_b8_bf16.json"):
    """Load a committed conv plan for the pipeline's forward batch (frames_per_forward x streams):
    the per-op kernel variants then do not depend on the batch, so pipelines with other forward
    batches compute bit-identical detections (the heuristic plan picks tiles by batch)."""
    with open(os.path.join(REPO, path)) as f:
        plan = json.load(f)["plan"]
    for m in pipe.models:
        m.load_plan(pipe.T * pipe.S, plan)


def test_pipelined_tracker_stream_matches_serial():
    """pipelined=True (tracker(t) on its own stream, overlapping detector(t+1), double-buffered
    detections) and inflight=2/3/4 (detector graphs in flight on their own streams) give exactly the
    serial pipeline's tracker state."""
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 4, 24
    runs = []
    # (pipelined, inflight, frames per forward): T > 1 is temporal batching (one forward of T
    # steps' frames); T = 5 leaves a partial forward for flush() at the end (24 = 4 x 5 + 4)
    for pipelined, inflight, tb in ((False, 1, 1), (True, 1, 1), (True, 2, 1), (True, 3, 1), (True, 4, 1),
                                    (True, 4, 2), (True, 2, 3), (True, 3, 5)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, frames_per_forward=tb)
        _plan_at_forward_batch(pipe)
        scenes = [P.synth.Scene(seed=40 + s, n_targets=16, n_frames=F) for s in range(S)]
        frames = torch.stack([sc.frames_torch(0, F, "cuda") for sc in scenes], 1)
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        for t in range(F):
            pipe.run(frames[t])
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        runs.append((rows.copy(), counts.copy(), stats.copy()))
    r0, c0, s0 = runs[0]
    for r1, c1, s1 in runs[1:]:
        np.testing.assert_array_equal(c0, c1)
        np.testing.assert_array_equal(s0, s1)
        for s in range(S):
            assert r0[s][: c0[s]].tobytes() == r1[s][: c1[s]].tobytes()


def test_prefetched_host_frames_match_device_frames():
    """Page-locked host frames through run(frames) (DMA on the slot stream), run(frames,
    next_frames=...) and prefetch() 1 and 3 steps ahead (the copy stream's staging ring) give
    exactly the tracker state of the same frames handed over in HBM; device frames prefetch too;
    frames other than the prefetched ones, or a prefetch beyond the staging ring, are refused."""
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 8, 20
    scenes = [P.synth.Scene(seed=60 + s, n_targets=16, n_frames=F) for s in range(S)]
    frames = torch.stack([sc.frames_torch(0, F, "cuda") for sc in scenes], 1).contiguous()
    host = frames.cpu().pin_memory()
    assert host[0].numel() >= pipeline.StreamPipeline.PULL_BYTES  # the DMA / staging path, not the pull kernel
    runs = []
    for mode in ("device", "direct", "next", "ahead1", "ahead3", "device_ahead2", "t2_ahead2", "t2_next"):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=True, inflight=4, frames_per_forward=2 if mode.startswith("t2") else 1)
        _plan_at_forward_batch(pipe)
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        src = frames if mode.startswith("device") else host
        depth = {"ahead1": 1, "ahead3": 3, "device_ahead2": 2, "t2_ahead2": 2}.get(mode, 0)
        for t in range(F):
            if mode in ("next", "t2_next"):
                pipe.run(src[t], next_frames=src[t + 1] if t + 1 < F else None)
            else:
                pipe.run(src[t])
            for u in range(t + 1 + pipe.n_prefetched, min(t + 1 + depth, F)):
                pipe.prefetch(src[u])
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        runs.append((rows.copy(), counts.copy(), stats.copy()))
        if mode == "ahead3":
            pipe.prefetch(host[0])
            with pytest.raises(ValueError):
                pipe.run(host[1])  # host[0] was prefetched for this step
            with pytest.raises(ValueError):
                for _ in range(pipe.nb + 8):
                    pipe.prefetch(host[0])
            pipe.sync()
    r0, c0, s0 = runs[0]
    assert c0.sum() > 0
    for r1, c1, s1 in runs[1:]:
        np.testing.assert_array_equal(c0, c1)
        np.testing.assert_array_equal(s0, s1)
        for s in range(S):
            assert r0[s][: c0[s]].tobytes() == r1[s][: c1[s]].tobytes()


def test_pulled_batch1_host_frames_match_device_frames():
    """Batch-1 page-locked frames (below PULL_BYTES: pulled onto the slot stream by
    yk_upload_pinned_async, four forwards in flight) give exactly the tracker state of the same
    frames handed over in HBM."""
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    F = 24
    sc = P.synth.Scene(seed=71, n_targets=24, n_frames=F)
    frames = sc.frames_torch(0, F, "cuda")[:, None].contiguous()  # [F, 1, H, W, 3]
    host = frames.cpu().pin_memory()
    assert host[0].numel() < pipeline.StreamPipeline.PULL_BYTES
    runs = []
    for src in (frames, host):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", 1, (512, 640), "fp32", seed=0, max_tracks=256,
                                       pipelined=True, inflight=4)
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        for t in range(F):
            pipe.run(src[t])
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        runs.append((rows.copy(), counts.copy(), stats.copy()))
    (r0, c0, s0), (r1, c1, s1) = runs
    assert c0.sum() > 0
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(s0, s1)
    assert r0[0][: c0[0]].tobytes() == r1[0][: c1[0]].tobytes()


def test_pipeline_with_global_motion_matches_serial():
    """StreamPipeline(tracker_policy=1, motion_method='optical_flow') -- the
    MotionCompensatedMultiTracker.update(dets, frame) loop with GlobalMotionDetector on the
    device -- gives the serial pipeline's tracker and motion-detector state when the motion
    detector reads each slot's frames on the tracker stream with forwards in flight.  The frames
    are camera pans over a textured world (tests/gmd_helpers.py) with whip pans that trigger the
    global reset branch."""
    from gmd_helpers import camera_sequence

    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S, F = 3, 20
    seqs = [camera_sequence(80 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()  # [F, S, H, W, 3]
    runs = []
    # inflight 4 is bench.py's CMC depth, 6 the depth round 4 saw differ (Lucas-Kanade end points
    # read beside forwards; the pipeline now runs the motion kernels in windows no forward overlaps)
    for pipelined, inflight in ((False, 1), (True, 1), (True, 3), (True, 4), (True, 6)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, tracker_policy=1,
                                       motion_method="optical_flow")
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        for t in range(F):
            pipe.run(frames[t])
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        motion, mstats = pipe.gmd.download()
        runs.append((rows.copy(), counts.copy(), stats.copy(), motion.copy(), mstats.copy()))
    r0, c0, s0, m0, ms0 = runs[0]
    assert int(ms0["reset_triggers"].sum()) > 0  # the whip pans reached the global reset branch
    for r1, c1, s1, m1, ms1 in runs[1:]:
        np.testing.assert_array_equal(c0, c1)
        np.testing.assert_array_equal(s0, s1)
        for f in m0.dtype.names:  # field by field, so a mismatch prints the values
            np.testing.assert_array_equal(m1[f], m0[f], err_msg=f"motion.{f}")
        for f in ms0.dtype.names:
            np.testing.assert_array_equal(ms1[f], ms0[f], err_msg=f"gmd stats.{f}")
        for s in range(S):
            assert r0[s][: c0[s]].tobytes() == r1[s][: c1[s]].tobytes()


def test_motion_windows_record_every_step_and_download_in_order():
    """Motion windows (pipelined tracker stream + motion detector): a wave's tracker steps are
    enqueued in its window, so the step hook and download_async of each step must still see that
    step's own tracker output.  Every step's recorded tracker rows at inflight 4 (a partial last
    wave included: 18 steps) equal the serial pipeline's, and the page-locked download of the last
    step equals the tracker's final state."""
    from gmd_helpers import camera_sequence
    from gpu_helpers import StepRecorder

    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    L = P._lib
    S, F = 2, 18
    seqs = [camera_sequence(60 + s, F, h=512, w=640, whip_at=(6, 12), n_targets=10)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()
    recs = []
    for pipelined, inflight in ((False, 1), (True, 4)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, tracker_policy=1,
                                       motion_method="optical_flow")
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        rec = StepRecorder(pipe, F)
        pipe.step_hook = rec
        rows_h = torch.empty(S * 256 * L.TRACK_OUT_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
        counts_h = torch.empty(S, dtype=torch.int32, pin_memory=True)
        stats_h = torch.empty(S * L.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
        for t in range(F):
            pipe.run(frames[t])
            if pipelined:
                pipe.download_async(rows_h, counts_h, stats_h)
        pipe.sync()
        recs.append(rec.host())
        if pipelined:
            rows, counts, _ = pipe.tracker.download()
            got = rows_h.numpy().view(L.TRACK_OUT_DTYPE).reshape(S, -1)
            np.testing.assert_array_equal(counts_h.numpy(), counts)
            for s in range(S):
                assert got[s, : counts[s]].tobytes() == rows[s, : counts[s]].tobytes()
    (d0, n0, r0, c0, s0), (d1, n1, r1, c1, s1) = recs
    np.testing.assert_array_equal(n0, n1)
    np.testing.assert_array_equal(c0, c1)
    for t in range(F):
        for s in range(S):
            assert r0[t, s, : c0[t, s]].tobytes() == r1[t, s, : c1[t, s]].tobytes(), (t, s)


def test_motion_windows_with_temporal_batching_match_serial():
    """Temporal batching inside motion windows (frames_per_forward T > 1 with the motion
    detector): a forward carries T steps' frames, the window runs the motion detector on each
    step's sub-batch in frame order, then the tracker steps.  The serial pipeline's tracker rows
    (every step, through the step hook), motion records and detector statistics are reproduced at
    T = 2 with 2 / 3 forwards in flight and at T = 3 (20 steps: a partial last forward), device
    frames and page-locked host frames prefetched ahead; download_async of each step hands back
    that step's output.  One committed plan at every forward batch (the per-op variants fix the
    detections' rounding)."""
    from gmd_helpers import camera_sequence
    from gpu_helpers import StepRecorder

    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    L = P._lib
    S, F = 3, 20
    seqs = [camera_sequence(70 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()  # [F, S, H, W, 3]
    host = frames.cpu().pin_memory()
    runs = []
    for pipelined, inflight, T, pinned in ((False, 1, 1, False), (True, 2, 2, False), (True, 3, 2, True),
                                           (True, 3, 3, False)):
        pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, tracker_policy=1,
                                       motion_method="optical_flow", frames_per_forward=T)
        _plan_at_forward_batch(pipe)
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        rec = StepRecorder(pipe, F)
        pipe.step_hook = rec
        rows_h = torch.empty(S * 256 * L.TRACK_OUT_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
        counts_h = torch.empty(S, dtype=torch.int32, pin_memory=True)
        stats_h = torch.empty(S * L.STATS_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
        for t in range(F):
            if pinned:  # this step's host frames, the next two steps' uploads issued ahead
                pipe.run(host[t])
                for u in range(t + 1 + pipe.n_prefetched, min(t + 3, F)):
                    pipe.prefetch(host[u])
            else:
                pipe.run(frames[t])
            if pipelined:
                pipe.download_async(rows_h, counts_h, stats_h)
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        if pipelined:  # the last step's page-locked copy is the tracker's final state
            got = rows_h.numpy().view(L.TRACK_OUT_DTYPE).reshape(S, -1)
            np.testing.assert_array_equal(counts_h.numpy(), counts)
            for s in range(S):
                assert got[s, : counts[s]].tobytes() == rows[s, : counts[s]].tobytes()
        motion, mstats = pipe.gmd.download()
        runs.append((rec.host(), stats.copy(), motion.copy(), mstats.copy(), (inflight, T)))
        del pipe
    (d0, n0, r0, c0, s0), st0, m0, ms0, _ = runs[0]
    assert int(ms0["reset_triggers"].sum()) > 0  # the whip pans reached the global reset branch
    for ((d1, n1, r1, c1, s1), st1, m1, ms1, cfg) in runs[1:]:
        np.testing.assert_array_equal(n0, n1, err_msg=str(cfg))
        np.testing.assert_array_equal(c0, c1, err_msg=str(cfg))
        np.testing.assert_array_equal(st0, st1, err_msg=str(cfg))
        for f in m0.dtype.names:
            np.testing.assert_array_equal(m1[f], m0[f], err_msg=f"motion.{f} {cfg}")
        for f in ms0.dtype.names:
            np.testing.assert_array_equal(ms1[f], ms0[f], err_msg=f"gmd stats.{f} {cfg}")
        for t in range(F):
            for s in range(S):
                assert r0[t, s, : c0[t, s]].tobytes() == r1[t, s, : c1[t, s]].tobytes(), (t, s, cfg)


def _pan_scene(seed, F, K=10):
    """A camera pan (tests/gmd_helpers.py, texture at 0.6 contrast) over K bright 18-px targets
    that move with the world plus their own drift: the planted detector sees ~2 boxes per
    target and nothing on the texture, the 50+ px/frame pans trigger the global reset branch,
    and the targets' screen jumps the per-track motion resets."""
    from gmd_helpers import camera_sequence

    frames, off = camera_sequence(seed, F, h=512, w=640, whip_at=(8, 16), n_targets=0)
    rng = np.random.default_rng(seed)
    pos, vel = rng.uniform([60, 60], [452, 580], (K, 2)), rng.normal(0, 1.5, (K, 2))
    out = (frames.astype(np.float32) * 0.6 + 20).astype(np.uint8)
    for f in range(F):
        for y, x in pos + vel * f - (off[f] - off[0]):
            y, x = int(y) % 480, int(x) % 600
            out[f, y:y + 18, x:x + 18] = 240
    return out


@pytest.mark.timeout(600)
def test_stream_pipeline_global_motion_fp32_matches_oracle_chain():
    """StreamPipeline(tracker_policy=1, motion_method='optical_flow') at fp32 -- device detector,
    device GlobalMotionDetector and the motion-reset tracker on the two-launch step -- against the
    oracle chain per stream and frame.  The detections of every step equal the torch-CPU
    detector's (oracle/detector_ref.py; counts identical, boxes / scores within 1e-4); the oracle
    tracker RefCMCMultiTracker(150, 1, 0.1).update(dets, frame) with its own
    RefGlobalMotionDetector (oracle/cmc_ref.py + oracle/gmd_ref.py) is fed the step's device
    detections (so a near-tie between two boxes of one target cannot move an association), and
    every tracker row is held to the motion-reset tests' bars (test_cmc_gpu.compare: decisions
    and counters identical, floats within 1e-9); global_resets / individual_resets /
    tracking_recoveries identical, global resets reached."""
    from oracle.cmc_ref import RefCMCMultiTracker
    from test_cmc_gpu import compare

    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    TR = P.tracker
    S, F = 2, 24
    seqs = [_pan_scene(90 + s, F) for s in range(S)]
    pipe = pipeline.StreamPipeline("yolov8s-small.yaml", S, (512, 640), "fp32", seed=0, max_tracks=256,
                                   tracker_policy=1, motion_method="optical_flow")
    ar = pipe.prog.ar
    ref = D.RefDetector(_layers(ar), pipe.prog.sd, P.arch.detect_strides(ar))
    refs = [RefCMCMultiTracker(150, 1, 0.1) for _ in range(S)]
    torch.set_num_threads(8)
    n_rows = 0
    for t in range(F):
        fr = [seqs[s][t] for s in range(S)]
        pipe.run(torch.from_numpy(np.stack(fr)).cuda())
        pipe.sync()
        rows, counts, stats = pipe.tracker.download()
        dd, dc = pipe.dets.cpu().numpy(), pipe.counts.cpu().numpy()
        want, _ = D.predict(ref, fr)
        for s in range(S):
            where = f"frame {t} stream {s}"
            w = want[s].numpy()
            assert int(dc[s]) == len(w), where
            np.testing.assert_allclose(dd[s, : dc[s], :4], w[:, :4], rtol=1e-4, atol=1e-3, err_msg=where)
            np.testing.assert_allclose(dd[s, : dc[s], 4], w[:, 4], rtol=1e-4, atol=1e-6, err_msg=where)
            dets = [[b[0], b[1], b[2], b[3], b[4]] for b in dd[s, : dc[s], :5]]
            rb = refs[s].update(dets, fr[s])
            ours = [TR._reset_fields(r, TR._row_to_dict(r, TR.track_id_of(r["track_num"]))) for r in rows[s, : counts[s]]]
            compare(ours, rb, where)
            for k in ("global_motion_events", "global_resets", "individual_resets", "tracking_recoveries"):
                assert int(stats[s][k]) == refs[s].stats[k], f"{where} {k}: {int(stats[s][k])} vs {refs[s].stats[k]}"
            n_rows += len(rb)
    assert n_rows > 200
    assert sum(r.stats["global_resets"] for r in refs) >= 2


def test_upload_pinned_async_copies_host_frames_exactly():
    """yk_upload_pinned_async (the pull kernel the pipeline uses for page-locked frames below
    StreamPipeline.PULL_BYTES): bit-exact copies of one and of eight 640x512 frames, a ragged
    16-byte multiple, and a refusal of pageable memory."""
    P = pkg()
    L = P._lib
    g = torch.Generator().manual_seed(3)
    for shape in ((1, 512, 640, 3), (8, 512, 640, 3), (7, 16)):
        src = torch.randint(0, 256, shape, dtype=torch.uint8, generator=g).pin_memory()
        dst = torch.zeros(shape, dtype=torch.uint8, device="cuda")
        L.check(L.lib().yk_upload_pinned_async(L.ptr(dst), L.ptr(src), src.numel(), L.current_stream(0)), "upload")
        torch.cuda.synchronize()
        assert torch.equal(dst.cpu(), src)
    pageable = torch.zeros(64, dtype=torch.uint8)
    dst = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(L.YKError):
        L.check(L.lib().yk_upload_pinned_async(L.ptr(dst), L.ptr(pageable), 64, L.current_stream(0)), "upload")


def test_run_refuses_next_frames_before_enqueuing_the_step():
    """run(frames, next_frames=...) that prefetch() would refuse -- no copy stream (inflight 1), or
    pageable (not page-locked) host frames -- raises before this step is enqueued: the
    step counter is unchanged and the same step then runs normally."""
    P = pkg()
    pipeline = importlib.import_module(P.__name__ + ".pipeline")
    S = 8
    sc = [P.synth.Scene(seed=90 + s, n_targets=8, n_frames=3) for s in range(S)]
    frames = torch.stack([x.frames_torch(0, 3, "cuda") for x in sc], 1).contiguous()
    pinned = frames.cpu().pin_memory()
    pageable = frames.cpu()
    assert pinned[0].numel() >= pipeline.StreamPipeline.PULL_BYTES
    for inflight, bad in ((1, pinned[2]), (4, pageable[2])):
        pipe = pipeline.StreamPipeline("yolov8n-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=128,
                                       pipelined=True, inflight=inflight)
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        pipe.run(frames[0])
        k0 = pipe._k
        with pytest.raises(ValueError):
            pipe.run(frames[1], next_frames=bad)
        assert pipe._k == k0
        pipe.run(frames[1])
        pipe.sync()
        assert pipe._k == (k0 + 1) % pipe.nb
