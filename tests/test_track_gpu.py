"""YOLO.track() (engine/model.py:559-613 + trackers/track.py:18-100) on the device -- detector
(detector.hip) then ByteTrack / BoT-SORT (bytetrack.hip) -- against the oracle chain: the
torch-CPU detector (oracle/detector_ref.py, conf 0.1 as track() sets it) feeding
oracle/bytetrack_ref.RefTracker (the reference's default lap assignment), frame by frame.

Bars: the same tracked rows in the same order; track ids, scores and classes exact; boxes
(Results.boxes.data, 7 columns [x1 y1 x2 y2 id conf cls] clipped to the frame) within 1e-4
relative of the frame size; Boxes.id / .is_track as upstream."""
import importlib

import numpy as np
import pytest
import torch

from conftest import pkg
from oracle import bytetrack_ref as R
from oracle import detector_ref as D

pytestmark = pytest.mark.gpu


def _layers(ar):
    return [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
            for Ly in ar.layers]


def _expected(ref_det, trk, frame):
    """track.py:86-100 on the oracle chain for one frame: Results (N, 6) -> tracked (M, 7)."""
    want, _ = D.predict(ref_det, [frame], conf=0.1)
    det = want[0].numpy()
    tracks = trk.update(R.Dets(det[:, :4], det[:, 4], det[:, 5]), frame)
    if len(tracks) == 0:
        return det
    out = tracks[:, :-1].astype(np.float32).copy()
    out[:, [0, 2]] = np.clip(out[:, [0, 2]], 0, frame.shape[1])
    out[:, [1, 3]] = np.clip(out[:, [1, 3]], 0, frame.shape[0])
    return out


@pytest.mark.parametrize("tracker", ["bytetrack.yaml", "botsort.yaml", "botsort-none"])
def test_yolo_track_persist_matches_oracle_chain(tracker):
    """for frame in video: model.track(frame, persist=True) -- 60 frames of a 24-target scene with
    occlusions; one tracker kept across calls.  botsort.yaml is the cfg default with its
    sparseOptFlow GMC (device gmd.hip / oracle gmc_ref.py, both fed the frame as track.py:93 does);
    botsort-none sets gmc_method: none (the identity warp)."""
    P = pkg()
    cfg = dict(R.BOTSORT_CFG if tracker.startswith("botsort") else R.BYTETRACK_CFG)
    if tracker == "botsort-none":
        cfg["gmc_method"] = "none"
    model = P.YOLO("yolov8s-small.yaml")
    ref_det = D.RefDetector(_layers(model.arch), model.state_dict, P.arch.detect_strides(model.arch))
    trk = R.RefTracker(cfg, ids=R.IdCounter())
    sc = P.synth.Scene(seed=11, n_targets=24, n_frames=61)
    torch.set_num_threads(8)
    n_tracked = 0
    ids = set()
    for t in range(60):
        frame = sc.frame(t)
        res = model.track(frame, persist=True, tracker=cfg, verbose=False)
        assert len(res) == 1
        got = res[0].boxes.data.cpu().numpy()
        exp = _expected(ref_det, trk, frame)
        assert got.shape == exp.shape, (t, got.shape, exp.shape)
        if exp.shape[1] == 7:
            assert res[0].boxes.is_track
            np.testing.assert_array_equal(got[:, 4], exp[:, 4], err_msg=f"frame {t}: track ids")
            np.testing.assert_array_equal(res[0].boxes.id.cpu().numpy(), exp[:, 4])
            n_tracked += len(exp)
            ids.update(exp[:, 4].tolist())
        np.testing.assert_allclose(got[:, -2:], exp[:, -2:], rtol=1e-4, atol=1e-6, err_msg=f"frame {t}: conf/cls")
        np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=0, atol=1e-4 * 640, err_msg=f"frame {t}: boxes")
    assert n_tracked > 300 and len(ids) >= 20


def test_yolo_track_list_source_resets_per_image_and_default_cfg():
    """A list of frames is one LoadPilAndNumpy batch whose paths are image{i}.jpg: without persist
    the tracker resets at every new path (track.py:90-93), so every frame starts new tracks (ids
    from 1); with persist the frames chain.  The plain call uses the cfg default (botsort.yaml
    with its sparseOptFlow GMC) and runs."""
    P = pkg()
    model = P.YOLO("yolov8s-small.yaml")
    sc = P.synth.Scene(seed=12, n_targets=16, n_frames=5)
    frames = [sc.frame(t) for t in range(4)]
    res0 = model.track(frames)  # defaults: botsort.yaml, GMC sparseOptFlow
    assert len(res0) == 4 and any(r.boxes.is_track for r in res0)
    res = model.track(frames, tracker="bytetrack.yaml")
    for r in res:
        if r.boxes.is_track:
            assert r.boxes.id.min().item() == 1  # fresh tracker per image (reset_id)
    res2 = P.YOLO("yolov8s-small.yaml").track(frames, tracker="bytetrack.yaml", persist=True)
    ref_det = D.RefDetector(_layers(model.arch), model.state_dict, P.arch.detect_strides(model.arch))
    trk = R.RefTracker(dict(R.BYTETRACK_CFG), ids=R.IdCounter())
    for f, r in zip(frames, res2):
        exp = _expected(ref_det, trk, f)
        got = r.boxes.data.cpu().numpy()
        assert got.shape == exp.shape
        np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=0, atol=1e-4 * 640)
        if exp.shape[1] == 7:
            np.testing.assert_array_equal(got[:, 4], exp[:, 4])
