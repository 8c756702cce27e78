"""The chain tests' near-tie accounting (gpu_helpers.dets_match / near_tie_boxes) on the CPU: a
detection list may differ from the oracle's only through near-ties, and the permutation it
reports maps the GPU's rows onto the oracle's."""
import numpy as np
import torch

from gpu_helpers import dets_match, near_tie_boxes


def _w():
    return np.array([[0, 0, 10, 10, .9], [20, 20, 30, 30, .8], [40, 40, 50, 50, .8]], np.float32)


def test_same_and_order_tie():
    w = _w()
    assert dets_match(w, w) == "same"
    g = w[[0, 2, 1]]  # equal scores in the other order
    assert dets_match(g, w) == "tie" and not dets_match.flip
    assert (w[dets_match.perm] == g).all()


def test_rejects_real_differences():
    w = _w()
    assert dets_match(w[:2], w) is None  # count
    g = w.copy()
    g[1, 0] += 5  # a moved box, no near-tie
    assert dets_match(g, w) is None
    w2 = w.copy()
    w2[2, 4] = 0.7  # distinct scores: the order is resolved, a swap is a failure
    assert dets_match(w2[[0, 2, 1]], w2) is None


def test_nms_near_tie_member_flip():
    w = _w()
    near = np.array([[20, 20, 30, 30], [24, 20, 34, 30]], np.float32)
    g = w.copy()
    g[1, :4] = [24, 20, 34, 30]
    assert dets_match(g, w, near) == "tie" and dets_match.flip
    assert dets_match(g, w, near[:1]) is None  # the kept box must itself be a pair member


def test_near_tie_boxes_pairs_overlapping_close_scores():
    # [5, A]: cx, cy, w, h, score; anchors 0/1 overlap with a 2e-6 score gap, 2 is far away
    y = torch.tensor([[100., 102., 300.], [100., 100., 300.], [40., 40., 40.], [40., 40., 40.],
                      [0.9966091, 0.9966071, 0.9966080]])
    nb = near_tie_boxes(y, (512, 640))
    assert nb.shape == (2, 4)
    assert len(near_tie_boxes(y, (512, 640), rel=1e-7)) == 0
