"""YOLO.predict (the ultralytics.YOLO surface, engine/model.py:498-557) against the oracle's
predict chain: the call's kwargs (conf, iou, max_det, classes, imgsz), a frame off the network
scale (LetterBox resize + scale_boxes), batched sources of mixed shapes, Results fields.
fp32 build; bar: boxes within 1e-4 relative (atol 1e-3 px), scores 1e-6."""
import importlib

import numpy as np
import pytest
import torch

from conftest import pkg
from oracle import detector_ref as D

pytestmark = pytest.mark.gpu


def _oracle(P, frames, conf, iou, max_det, imgsz):
    A = P.arch
    ar = A.parse_arch(A.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 0)
    from test_detector_gpu import layer_list

    ref = D.RefDetector(layer_list(ar), sd, A.detect_strides(ar))
    torch.set_num_threads(8)
    im = D.preprocess(frames, imgsz)
    y, _ = ref.forward(im)
    res = D.non_max_suppression(y, conf, iou, max_det)
    return [D.scale_clip(p, im.shape[2:], frames[0].shape[:2]) for p in res]


def _close(r, ref):
    got = r.boxes.data.cpu().numpy()
    assert got.shape[0] == len(ref), (got.shape, len(ref))
    np.testing.assert_allclose(got[:, :4], ref[:, :4].numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(got[:, 4], ref[:, 4].numpy(), rtol=1e-4, atol=1e-6)


def _iou_np(a, b):
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:4], b[None, :, 2:4])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (aa[:, None] + ab[None] - inter)


def test_predict_kwargs_match_oracle():
    P = pkg()
    model = P.YOLO("yolov8s-small.yaml", dtype="fp32")
    sc = P.synth.Scene(seed=21, n_targets=30, n_frames=3)
    frames = [sc.frame(0), sc.frame(1)]
    for conf, iou, max_det in ((0.25, 0.7, 300), (0.4, 0.5, 300), (0.25, 0.7, 5)):
        res = model(frames, conf=conf, iou=iou, max_det=max_det, verbose=False)
        refs = _oracle(P, frames, conf, iou, max_det, 640)
        assert len(res) == 2
        for r, ref in zip(res, refs):
            _close(r, ref)
            assert r.orig_shape == (512, 640) and set(r.speed) == {"preprocess", "inference", "postprocess"}
        if max_det == 5:
            assert all(len(r.boxes) == 5 for r in res)
    # classes= filters before NMS (nms.py:128-132): single-class head -> all or nothing
    assert len(model(frames[0], classes=[0])[0].boxes) == len(model(frames[0])[0].boxes) > 0
    assert len(model(frames[0], classes=[1])[0].boxes) == 0
    # half=True: the fp16 build (AutoBackend(fp16=True) -> model.half()), its own engine; the
    # detections agree with the fp32 ones to fp16 rounding
    rh = model(frames, half=True, verbose=False)
    assert any(k[-1] == "fp16" for k in model._engines)
    for r16, r32 in zip(rh, model(frames, verbose=False)):
        a, b = r16.boxes.data.cpu().numpy(), r32.boxes.data.cpu().numpy()
        assert abs(len(a) - len(b)) <= max(2, len(b) // 10)
        if len(b):
            iou = _iou_np(b[:, :4], a[:, :4])
            assert (iou.max(1) > 0.5).mean() >= 0.95
    with pytest.raises(AssertionError):
        model(frames[0], conf=1.5)


def test_predict_letterboxed_and_mixed_shapes_match_oracle():
    P = pkg()
    model = P.YOLO("yolov8s-small.yaml", dtype="fp32")
    big = P.synth.Scene(seed=22, n_targets=24, n_frames=2, width=1280, height=720).frame(0)
    small = P.synth.Scene(seed=23, n_targets=12, n_frames=2).frame(0)
    res = model([big, small], imgsz=640, verbose=False)
    _close(res[0], _oracle(P, [big], 0.25, 0.7, 300, 640)[0])
    _close(res[1], _oracle(P, [small], 0.25, 0.7, 300, 640)[0])
    assert res[0].orig_shape == (720, 1280) and res[1].orig_shape == (512, 640)
    xyxy = res[0].boxes.xyxy.cpu().numpy()
    assert (xyxy[:, [0, 2]] <= 1280).all() and (xyxy[:, [1, 3]] <= 720).all() and (xyxy >= 0).all()
