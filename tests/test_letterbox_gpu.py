"""GPU parity of the LetterBox resize path (letterbox_kernel in csrc/detector.hip): frames off the
network scale (1920x1080, 1280x1024 and 800x600 at imgsz 640, 400x300 upscaled) are resized on
the device exactly as oracle/letterbox_ref.py restates cv2.resize INTER_LINEAR (bit-identical
uint8 canvases; parity with cv2 itself unpinned, no cv2 here), and the fp32 detections match
the oracle's predict (boxes mapped back by scale_boxes with gain != 1) to 1e-4."""
import importlib

import numpy as np
import pytest
import torch

from conftest import pkg
from oracle import detector_ref as D
from oracle.letterbox_ref import letterbox

pytestmark = pytest.mark.gpu


def _layers(ar):
    return [(Ly.i, Ly.f, Ly.kind, {**Ly.args, **({"c": int(Ly.c2 * 0.5)} if Ly.kind == "C2f" else {})})
            for Ly in ar.layers]


@pytest.mark.parametrize("hw", [(1080, 1920), (1024, 1280), (600, 800), (300, 400)])
def test_letterbox_resize_and_detections_match_oracle(hw):
    P = pkg()
    A = importlib.import_module(P.__name__ + ".arch")
    W = importlib.import_module(P.__name__ + ".weights")
    M = importlib.import_module(P.__name__ + ".model")
    ar = A.parse_arch(A.load_model_dict("yolov8-small.yaml"))
    sd = W.synthetic_state_dict(ar, 0)
    B = 2
    sc = P.synth.Scene(seed=3, n_targets=24, n_frames=B + 1, height=hw[0], width=hw[1])
    frames = [sc.frame(t) for t in range(B)]
    dm = M.DeviceModel(M.Program(ar, sd, hw[0], hw[1], 640, B, "fp32"))
    assert dm.prog.lb["mode"] != 0
    ft = torch.from_numpy(np.stack(frames)).cuda()
    dets, counts = dm.detect(ft, 0.25, 0.7, 300)
    torch.cuda.synchronize()
    canvas = dm.letterboxed(B)
    for b in range(B):
        np.testing.assert_array_equal(canvas[b], letterbox(frames[b]))
    torch.set_num_threads(8)
    ref = D.RefDetector(_layers(ar), sd, A.detect_strides(ar))
    want, _ = D.predict(ref, frames, 0.25, 0.7, 300, 640)
    total = 0
    for b in range(B):
        n = int(counts[b])
        assert n == len(want[b])
        total += n
        got = dets[b, :n].cpu()
        np.testing.assert_allclose(got[:, :4].numpy(), want[b][:, :4].numpy(), rtol=1e-4, atol=2e-3)
        np.testing.assert_allclose(got[:, 4].numpy(), want[b][:, 4].numpy(), rtol=1e-4, atol=1e-6)
    assert total > 0
