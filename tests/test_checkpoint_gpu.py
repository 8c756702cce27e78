"""§8f-2 on the GPU: YOLO("best.pt") -- an ultralytics-style checkpoint (pickled DetectionModel,
fp16 weights, the parsed YAML on model.yaml; written by tests/ckpt_helpers.py since the reference
ships none) read without ultralytics and without executing the pickle (checkpoint.py,
nn/tasks.py:1404-1521: load_checkpoint ... .float()) -- predicts what the oracle predicts when it
is built from the same state dict (fp16 -> fp32, as the reference's .float()).  Scale n is what
the reference's training run resolved to (small_target_detection/yolov8_small_aircraft/args.yaml:3,
yolov8-small.yaml); scale s is BASELINE's "YOLOv8s+P2"."""
import numpy as np
import pytest
import torch

from ckpt_helpers import write_checkpoint
from conftest import pkg
from oracle import detector_ref as D

pytestmark = pytest.mark.gpu


def _layers(ar):
    return [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
            for Ly in ar.layers]


@pytest.mark.parametrize("yaml_name,scale", [("yolov8-small.yaml", "n"), ("yolov8s-small.yaml", "s")])
def test_yolo_best_pt_predict_matches_oracle(tmp_path, yaml_name, scale):
    P = pkg()
    y = P.arch.load_model_dict(yaml_name)
    ar = P.arch.parse_arch(y)
    assert ar.scale == scale
    sd = P.weights.synthetic_state_dict(ar, 5)
    path = str(tmp_path / "best.pt")
    write_checkpoint(path, ar, y, sd, half=True)
    model = P.YOLO(path)  # no dtype: the drop-in default (fp32)
    assert model.dtype == "fp32" and model.arch.scale == scale and model.ckpt_meta["version"] == "8.3.193"
    sd32 = {k: (v.half().float() if v.is_floating_point() else v) for k, v in sd.items()}
    ref = D.RefDetector(_layers(ar), sd32, P.arch.detect_strides(ar))
    sc = P.synth.Scene(seed=8, n_targets=24, n_frames=3)
    frames = [sc.frame(t) for t in range(2)]
    res = model(frames, verbose=False)
    torch.set_num_threads(8)
    want, _ = D.predict(ref, frames)
    n_boxes = 0
    for r, w in zip(res, want):
        got = r.boxes.data.cpu().numpy()
        w = w.numpy()
        assert got.shape == w.shape
        np.testing.assert_allclose(got[:, :4], w[:, :4], rtol=1e-4, atol=1e-3)
        np.testing.assert_allclose(got[:, 4], w[:, 4], rtol=1e-4, atol=1e-6)
        n_boxes += len(w)
    assert n_boxes > 0
