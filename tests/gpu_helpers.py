"""GPU test plumbing: record a pipelined StreamPipeline's per-step outputs without
synchronising it, and compare track dicts against the oracle."""
import ctypes as C
import os

import numpy as np
import torch

from conftest import pkg

_hip = None


def _hip_rt():
    """torch's bundled HIP runtime (the one libyk.so and torch share)."""
    global _hip
    if _hip is None:
        _hip = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip.hipMemcpyAsync.restype = C.c_int
    return _hip


def d2d_async(dst: int, src: int, nbytes: int, stream) -> None:
    rc = _hip_rt().hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), nbytes, 3, C.c_void_p(stream.cuda_stream))
    assert rc == 0, f"hipMemcpyAsync failed: {rc}"


class StepRecorder:
    """StreamPipeline.step_hook that copies, in stream order, every step's detections (on the
    detector stream) and the tracker's output rows / counts / stats (on the tracker stream)
    into per-step device history buffers; host() downloads them after the run."""

    def __init__(self, pipe, n_steps: int):
        L = pkg()._lib
        self.L = L
        S, T = pipe.S, pipe.tracker.max_tracks
        dev = torch.device("cuda", pipe.device)
        self.n, self.t = n_steps, 0
        self.dets = torch.zeros((n_steps, S, pipe.max_det, 6), dtype=torch.float32, device=dev)
        self.counts = torch.zeros((n_steps, S), dtype=torch.int32, device=dev)
        self.row_bytes = S * T * L.TRACK_OUT_DTYPE.itemsize
        self.stat_bytes = S * L.STATS_DTYPE.itemsize
        self.rows = torch.zeros((n_steps, self.row_bytes), dtype=torch.uint8, device=dev)
        self.tcounts = torch.zeros((n_steps, S), dtype=torch.int32, device=dev)
        self.stats = torch.zeros((n_steps, self.stat_bytes), dtype=torch.uint8, device=dev)
        self.S, self.T = S, T

    def __call__(self, pipe, k, det_stream, trk_stream):
        t = self.t
        assert t < self.n, "more steps than the recorder holds"
        dets, counts = pipe.step_outputs(k)
        with torch.cuda.stream(det_stream):
            self.dets[t].copy_(dets)
            self.counts[t].copy_(counts)
        rows, counts, stats = pipe.tracker.device_outputs()
        d2d_async(self.rows[t].data_ptr(), rows, self.row_bytes, trk_stream)
        d2d_async(self.tcounts[t].data_ptr(), counts, self.S * 4, trk_stream)
        d2d_async(self.stats[t].data_ptr(), stats, self.stat_bytes, trk_stream)
        self.t += 1

    def host(self):
        torch.cuda.synchronize()
        n = self.t
        rows = self.rows[:n].cpu().numpy().view(self.L.TRACK_OUT_DTYPE).reshape(n, self.S, self.T)
        stats = self.stats[:n].cpu().numpy().view(self.L.STATS_DTYPE).reshape(n, self.S)
        return (self.dets[:n].cpu().numpy(), self.counts[:n].cpu().numpy(), rows, self.tcounts[:n].cpu().numpy(),
                stats)


def track_dicts(rows, n):
    P = pkg()
    return [P.tracker._row_to_dict(r, P.tracker.track_id_of(r["track_num"])) for r in rows[:n]]


def decisions(tracks):
    """The association decisions of one frame: (track_id, status, age, hits, tsu) per output."""
    return [(d["track_id"], d["status"], d["age"], d["hits"], d["time_since_update"]) for d in tracks]


def assign_margin(iou, thr):
    """Conditioning of one frame's greedy association (ref_greedy_assign): the smallest gap between
    a taken pair's IoU and the best still-free pair it beat in its row or column, and between any
    IoU and the gate thr.  Two chains whose IoUs differ by less than this make the same decisions;
    a strict chain comparison is only a parity test on inputs where it is well above the chains'
    IoU spread (~1e-6 for the fp32 detector)."""
    iou = np.asarray(iou, np.float64)
    if iou.size == 0:
        return np.inf
    m = float(np.min(np.abs(iou - thr)))
    di, ti = np.where(iou >= thr)
    if not len(di):
        return m
    v = iou[di, ti]
    order = np.argsort(-v, kind="stable")
    used_d, used_t = set(), set()
    for n, k in enumerate(order):
        d, t = di[k], ti[k]
        if d in used_d or t in used_t:
            continue
        for k2 in order[n + 1:]:  # the next free competitor sharing the row or the column
            d2, t2 = di[k2], ti[k2]
            if (d2 == d or t2 == t) and d2 not in used_d and t2 not in used_t:
                m = min(m, float(v[k] - v[k2]))
                break
        used_d.add(d)
        used_t.add(t)
    return m


def near_tie_boxes(pred: torch.Tensor, hw, conf: float = 0.25, iou: float = 0.7, rel: float = 1e-5):
    """NMS near-ties of one image's Detect output [5, A]: candidates (score > conf) that overlap
    another candidate at IoU > iou (so NMS keeps exactly one of the two) with scores within `rel`
    of each other.  Two fp32 convolution implementations that differ only in summation order
    (activations within ~3e-6 of each other, max-normalised) may keep either member of such a
    pair; returns every member's box clipped to the frame (xyxy, float32 [N, 4])."""
    s = pred[4]
    idx = torch.nonzero(s > conf).flatten()
    if idx.numel() < 2:
        return np.zeros((0, 4), np.float32)
    b = pred[:4, idx].T
    xy = torch.cat((b[:, :2] - b[:, 2:] / 2, b[:, :2] + b[:, 2:] / 2), 1)
    lt = torch.maximum(xy[:, None, :2], xy[None, :, :2])
    rb = torch.minimum(xy[:, None, 2:], xy[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    area = (xy[:, 2] - xy[:, 0]) * (xy[:, 3] - xy[:, 1])
    ov = inter / (area[:, None] + area[None] - inter) > iou
    sc = s[idx]
    close = (sc[:, None] - sc[None]).abs() <= rel * torch.maximum(sc[:, None], sc[None])
    m = ov & close
    m.fill_diagonal_(False)
    xy = xy[m.any(1)]
    H, W = hw
    xy[:, 0::2] = xy[:, 0::2].clamp(0, W)
    xy[:, 1::2] = xy[:, 1::2].clamp(0, H)
    return xy.numpy().astype(np.float32)


def dets_match(got, want, near=None, rel: float = 1e-5):
    """Detections [N, >=5] of the GPU against the oracle's for one image, under the fp32 bars.
    Returns "same" (row by row within 1e-4 / atol 1e-3 px, scores 1e-4), "tie" (equal only up to
    near-ties: a row out of place sits among oracle rows whose scores are within `rel` of its own
    -- the score order is unresolved at fp32 resolution -- or a differing box is a member of an
    oracle NMS near-tie pair in `near`, see near_tie_boxes), or None.  After a call,
    dets_match.perm[j] is the oracle row GPU row j matched and dets_match.flip says whether an NMS
    near-tie kept the other member of a pair (otherwise the rows differ only in order)."""
    def close(a, b):
        return bool(np.all(np.abs(a[:4] - b[:4]) <= 1e-4 * np.abs(b[:4]) + 1e-3)) and \
            abs(float(a[4]) - float(b[4])) <= 1e-4 * abs(float(b[4])) + 1e-6

    def member(box):
        return near is not None and len(near) > 0 and \
            bool(np.any(np.all(np.abs(near - box[:4]) <= 1e-4 * np.abs(box[:4]) + 1e-3, axis=1)))

    n = len(want)
    dets_match.perm, dets_match.flip = np.arange(n), False
    if len(got) != n:
        return None
    if all(close(g, w) for g, w in zip(got, want)):
        return "same"
    for i in range(n):  # every differing position is explained by a near-tie
        if not close(got[i], want[i]):
            peers = np.abs(want[:, 4] - want[i, 4]) <= rel * abs(float(want[i, 4]))
            if peers.sum() < 2 and not (member(want[i]) and member(got[i])):
                return None
    used = np.zeros(n, bool)  # and the two sets agree (an NMS near-tie may swap a pair's member)
    perm, flip = np.zeros(n, int), False
    for i in range(n):
        j = next((j for j in range(n) if not used[j] and close(got[j], want[i])), None)
        if j is None:
            j = next((j for j in range(n) if not used[j] and member(got[j]) and member(want[i])
                      and abs(float(got[j, 4]) - float(want[i, 4])) <= rel * abs(float(want[i, 4]))), None)
            flip = True
        if j is None:
            return None
        used[j] = True
        perm[j] = i
    dets_match.perm, dets_match.flip = perm, flip  # GPU row j is oracle row perm[j]
    return "tie"


def resync_rows(got, want, perm):
    """The oracle chain's input after a near-tie frame (dets_match == "tie"): the oracle's rows in
    the GPU's order, except that a row the GPU kept instead of the oracle's pair member (an NMS
    near-tie flip) is the GPU's own row -- so the oracle chain continues on the boxes the GPU
    chain follows and every later frame's decisions can still be compared.  Also returns the
    flips as (oracle row, GPU row) pairs."""
    rows, flips = [], []
    for j in range(len(got)):
        w = want[perm[j]]
        same = bool(np.all(np.abs(got[j, :4] - w[:4]) <= 1e-4 * np.abs(w[:4]) + 1e-3))
        rows.append(w if same else got[j])
        if not same:
            flips.append((w, got[j]))
    return np.asarray(rows, np.float32).reshape(-1, want.shape[1]), flips


def score_ties(pred: torch.Tensor, conf: float = 0.25) -> int:
    """Exact duplicate scores among the NMS candidates (score > conf) of one image's Detect
    output [5, A]: non_max_suppression's scores.sort (utils/nms.py:264) is unstable on them."""
    s = pred[4][pred[4] > conf]
    return int(s.numel() - torch.unique(s).numel())


def lost_conf_spread(track, delta: float, samples: int = 8, seed: int = 0) -> float:
    """How far a lost track's reported confidence (get_lost_prediction -> long_term_predict,
    kf.py:205-247, 319-333) moves when every entry of its velocity history moves by ~delta
    (Gaussian, per component): the conditioning of that confidence.  Through the direction
    statistics (arctan2 of near-zero velocities) and the 0.3 / 0.5 thresholds a confidence can
    swing by far more than its inputs; two fp32 chains whose velocities differ by delta cannot be
    held closer than this.  `track` is an oracle RefTrack; nothing of it is modified."""
    import copy
    from collections import deque

    rng = np.random.default_rng(seed)
    _, c0 = copy.deepcopy(track).get_lost_prediction()
    spread = 0.0
    for _ in range(samples):
        t2 = copy.deepcopy(track)
        t2.velocity_history = deque([np.asarray(v, np.float64) + rng.normal(0.0, delta, 2) for v in track.velocity_history],
                                    maxlen=track.velocity_history.maxlen)
        _, c = t2.get_lost_prediction()
        spread = max(spread, abs(float(c) - float(c0)))
    return spread
