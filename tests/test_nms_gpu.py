"""nms_kernel (csrc/detector.hip) on GIVEN boxes through yk_nms, held to TorchNMS.nms
(ultralytics/utils/nms.py:237-304, restated in oracle/detector_ref.torch_nms with a stable sort)
and to the golden keep lists of tests/golden/nms.npz -- including SURVEY §8c's quirk-C known
answer [A, B, C] -- on every size path of the kernel (one-wave greedy loop <= 256, LDS bitmask
<= 512, LDS sort <= 2,048, global-memory sort above), with exact score ties, NaN scores and
coordinates and zero-area boxes; plus the device error flag for corrupt candidate rows."""
import importlib
import os
import sys

import numpy as np
import pytest
import torch

from conftest import pkg
from oracle import detector_ref as D

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402

pytestmark = pytest.mark.gpu

_DM = {}


def _model(max_det=1024):
    """YOLOv8n+P2 fp32 at 640x512 (27,200 candidate slots per image), only its NMS is used."""
    if max_det not in _DM:
        P = pkg()
        M = importlib.import_module(P.__name__ + ".model")
        ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8-small.yaml"))
        sd = P.weights.synthetic_state_dict(ar, 0)
        _DM[max_det] = M.DeviceModel(M.Program(ar, sd, 512, 640, 640, 2, "fp32", max_det))
    return _DM[max_det]


def _run(boxes, scores, thr, max_det=1024):
    dm = _model(max_det if max_det > 300 else 1024)
    n = len(boxes)
    rows = np.zeros((1, max(n, 1), 5), np.float32)
    rows[0, :n, :4] = boxes
    rows[0, :n, 4] = scores
    dets, cnt, keep = dm.nms(torch.from_numpy(rows).cuda(), torch.tensor([n], dtype=torch.int32).cuda(), thr, max_det)
    torch.cuda.synchronize()
    k = int(cnt[0])
    return dets[0, :k].cpu().numpy(), keep[0, :k].cpu().numpy()


def _clip(b):
    out = b.copy()
    out[:, [0, 2]] = np.clip(out[:, [0, 2]], 0, 640)
    out[:, [1, 3]] = np.clip(out[:, [1, 3]], 0, 512)
    return out


@pytest.mark.parametrize("case", range(7))
def test_nms_kernel_matches_golden_keep_lists(case):
    """Every tests/golden/nms.npz case bit-exact: keep order, kept rows (scale_boxes / clip of the
    input rows at gain 1, pad 0), scores.  Case 6 is the quirk-C KAT: A, then B and C, which
    overlap each other but not A, are all kept (standard NMS would drop C)."""
    boxes, scores, thr = G.nms_inputs()[case]
    want = G.load("nms")[f"keep{case}"]
    dets, keep = _run(boxes, scores, thr)
    np.testing.assert_array_equal(keep, want)
    np.testing.assert_array_equal(dets[:, :4], _clip(boxes[want]))
    np.testing.assert_array_equal(dets[:, 4], scores[want])
    if case == 6:
        assert keep.tolist() == [0, 1, 2]


def _edge_set(n, seed):
    """n boxes in a 640x512 field: clusters of 3-8 jittered boxes (every box overlaps its cluster,
    so the greedy loop suppresses instead of taking the early exit at the first isolated box), exact
    score ties (scores from 5 levels), a NaN score, a box with a NaN corner, and two identical
    zero-area boxes (union 0 -> IoU 0/0), all placed inside clusters."""
    rng = np.random.default_rng(seed)
    n_cl = max(n // 5, 1)
    centers = rng.uniform(20, 620, (n_cl, 2))
    sizes = rng.uniform(10, 60, (n_cl, 2))
    idx = rng.integers(0, n_cl, n)
    c = centers[idx] + rng.normal(0, 2.5, (n, 2))
    wh = sizes[idx] * rng.uniform(0.8, 1.2, (n, 2))
    b = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32)
    s = rng.choice(np.float32([0.3, 0.45, 0.6, 0.75, 0.9]), n).astype(np.float32)
    if n >= 8:
        s[3] = np.nan
        b[5, 2] = np.nan
        x0, y0 = float(b[0, 0]), float(b[0, 1])
        b[6] = [x0 + 1, y0 + 1, x0 + 1, y0 + 9]  # zero width, inside box 0's cluster
        b[7] = b[6]
        s[6] = s[7] = np.float32(0.3)  # late in the order: a zero-area kept box overlaps nothing (early exit)
    if n >= 16:
        s.view(np.uint32)[9] = 0xFFC00000  # a NaN with the sign bit set: torch still sorts it first
    return b, s


@pytest.mark.parametrize("n", [1, 8, 40, 200, 400, 1500, 3000])
@pytest.mark.parametrize("max_det,thr", [(300, 0.7), (1024, 0.7), (1024, 0.3)])
def test_nms_kernel_edge_cases_every_path(n, max_det, thr):
    """Ties (stable: input order), NaN scores of either sign (sorted first, as torch's sort puts
    every NaN), NaN corner
    (its IoU is NaN: suppressed by `iou <= thr` being false, never counted as no-overlap), degenerate
    boxes (0/0 IoU), and the max_det cut -- against torch_nms + [:max_det] on every size path."""
    boxes, scores = _edge_set(n, seed=n)
    want = D.torch_nms(torch.from_numpy(boxes), torch.from_numpy(scores), thr).numpy()[:max_det]
    dets, keep = _run(boxes, scores, thr, max_det)
    np.testing.assert_array_equal(keep, want)
    np.testing.assert_array_equal(dets[:, 4], scores[want])


def test_nms_early_exit_counter_and_corrupt_candidates_flag():
    """yk_model_nms_stats counts images whose greedy loop took the :291-296 early exit (the quirk-C
    case does, a set where every box overlaps the next does not).  A candidate row whose anchor
    field lies outside [0, n_anchors) -- what the round-2 graph-replay race produced -- no longer
    indexes outside the kernel's tables: that image's count is 0, and the next call on the model
    (or yk_model_check) reports YK_ERR_STATE once; both NMS size paths."""
    from gpu_helpers import d2d_async

    P = pkg()
    L = P._lib
    dm = _model()
    dm.nms_stats(reset=True)
    boxes, scores, thr = G.nms_inputs()[6]
    _run(boxes, scores, thr)
    chain = np.array([[0, 0, 10, 10], [5, 0, 15, 10], [10, 0, 20, 10]], np.float32)
    _run(chain, np.float32([0.9, 0.8, 0.7]), 0.99)  # each box overlaps the next: no early exit
    early, images = dm.nms_stats(reset=True)
    assert (early, images) == (1, 2)
    import ctypes as C

    cand, cnt = C.c_void_p(), C.c_void_p()
    L.check(L.lib().yk_model_candidates(dm.handle, C.byref(cand), C.byref(cnt)), "yk_model_candidates")
    A = dm.prog.n_anchors
    for n in (100, 1200):  # the <= 512 (LDS) and the > 512 NMS paths
        b, s = _edge_set(n, seed=7)
        _run(b, s, 0.7)  # loads n valid candidate rows into the model's candidate buffer
        bad = torch.tensor([[1.0, 1.0, 5.0, 5.0, 0.5, 0.0]], dtype=torch.float32, device="cuda")
        bad.view(torch.int32)[0, 5] = A + 17  # anchor index past n_anchors
        d2d_async(cand.value + 4 * 6 * 3, bad.data_ptr(), 24, torch.cuda.current_stream())
        dets, k, _ = dm.nms_candidates(1, 0.7, 300)
        torch.cuda.synchronize()
        assert int(k[0]) == 0
        with pytest.raises(L.YKError) as e:
            dm.check()
        assert e.value.status == L.YK_ERR_STATE and "anchor" in str(e.value)
        dm.check()  # reported once
        _, keep = _run(b, s, 0.7)  # the model works again
        assert len(keep) > 0
