"""Device ByteTrack / BoT-SORT (csrc/bytetrack.hip via yk_bt_*) against the numpy + scipy
restatement of ultralytics/trackers (oracle/bytetrack_ref.py), frame by frame.

Bar: the same rows in the same order, track ids / cls / idx / scores identical, boxes within
1e-3 px (float64 state differing from numpy's BLAS by an ulp, cast to float32)."""
import importlib

import numpy as np
import pytest

from bt_helpers import scenario
from conftest import pkg
from oracle import bytetrack_ref as R


def _bt():
    return importlib.import_module(pkg().__name__ + ".bytetrack")


def _compare(got, exp, where):
    assert got.shape == exp.shape, f"{where}: {got.shape} rows vs oracle {exp.shape}"
    if exp.size == 0:
        return
    np.testing.assert_array_equal(got[:, 4], exp[:, 4], err_msg=f"{where}: track ids")
    np.testing.assert_array_equal(got[:, 5:8], exp[:, 5:8], err_msg=f"{where}: score / cls / idx")
    np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-6, atol=1e-3, err_msg=f"{where}: boxes")


class _OrderProbe:
    """Counts, per assignment the oracle makes: scipy branch -- unmatched lists the reference
    iterates in a non-ascending (CPython frozenset) order, the cases the device's set-order
    simulation decides; lap branch -- assignments whose kept matches differ from the scipy
    branch's on the same cost matrix, the cases only the lapjv problem decides."""

    def __init__(self, monkeypatch):
        self.nonasc = self.lap_differs = 0
        orig = R.linear_assignment

        def wrapped(cost, thresh, use_lap=True):
            m, ua, ub = orig(cost, thresh, use_lap)
            if use_lap:
                ms = orig(cost, thresh, False)[0]
                self.lap_differs += sorted(map(tuple, np.asarray(m).reshape(-1, 2).tolist())) != \
                    sorted(map(tuple, np.asarray(ms).reshape(-1, 2).tolist()))
            else:
                self.nonasc += (list(ua) != sorted(ua)) + (list(ub) != sorted(ub))
            return m, ua, ub

        monkeypatch.setattr(R, "linear_assignment", wrapped)


@pytest.mark.gpu
@pytest.mark.parametrize("use_lap", [True, False], ids=["lap", "scipy"])
@pytest.mark.parametrize("kind", ["bytetrack", "botsort"])
def test_batched_streams_match_oracle(kind, use_lap, monkeypatch):
    probe = _OrderProbe(monkeypatch)
    BT = _bt()
    S, F = 3, 90
    cfg = dict(R.BOTSORT_CFG if kind == "botsort" else R.BYTETRACK_CFG)
    dev = BT.BatchedTracker(cfg, n_streams=S, max_tracks=256, max_dets=128, use_lap=use_lap)
    ids = R.IdCounter()
    refs = [R.RefTracker(cfg, ids=ids, use_lap=use_lap) for _ in range(S)]
    seqs = [scenario(20 + s, n_targets=36, n_frames=F) for s in range(S)]
    n_rows = n_new_ids = 0
    for f in range(F):
        per = [seqs[s][f] for s in range(S)]
        dev.step([np.c_[x, c, k] for x, c, k in per])
        got = dev.download()
        for s in range(S):
            exp = refs[s].update(R.Dets(*per[s]))
            _compare(got[s], exp, f"{kind} frame {f + 1} stream {s}")
            n_rows += len(exp)
    n_new_ids = ids.count
    assert n_rows > 1500 and n_new_ids > 150  # the sequences exercise births, losses and re-finds
    if use_lap:
        print("lap assignments that differ from the scipy branch:", probe.lap_differs)
    else:
        assert probe.nonasc > 20, probe.nonasc  # ... and set-ordered unmatched lists


@pytest.mark.gpu
@pytest.mark.parametrize("use_lap", [True, False], ids=["lap", "scipy"])
@pytest.mark.parametrize("kind", ["bytetrack", "botsort"])
def test_dense_crowd_matches_oracle(kind, use_lap, monkeypatch):
    """Many targets in a small field (large connected components in the assignment graph)."""
    probe = _OrderProbe(monkeypatch)
    BT = _bt()
    S, F = 2, 60
    cfg = dict(R.BOTSORT_CFG if kind == "botsort" else R.BYTETRACK_CFG)
    dev = BT.BatchedTracker(cfg, n_streams=S, max_tracks=512, max_dets=256, use_lap=use_lap)
    ids = R.IdCounter()
    refs = [R.RefTracker(cfg, ids=ids, use_lap=use_lap) for _ in range(S)]
    seqs = [scenario(40 + s, n_targets=110, n_frames=F, width=640.0, height=480.0, groups=12) for s in range(S)]
    for f in range(F):
        per = [seqs[s][f] for s in range(S)]
        dev.step([np.c_[x, c, k] for x, c, k in per])
        got = dev.download()
        for s in range(S):
            _compare(got[s], refs[s].update(R.Dets(*per[s])), f"{kind} dense frame {f + 1} stream {s}")
    if use_lap:
        assert probe.lap_differs > 0, "the crowd never separates the lap branch from the scipy one"
    else:
        assert probe.nonasc > 10


@pytest.mark.gpu
def test_single_stream_facade_and_reset():
    BT = _bt()
    trk = BT.BYTETracker(dict(BT.BYTETRACK_DEFAULTS), frame_rate=30, max_tracks=256, max_dets=128)
    ref = R.RefTracker(dict(R.BYTETRACK_CFG))
    seq = scenario(7, n_targets=20, n_frames=40)
    for rnd in range(2):
        for f, (x, c, k) in enumerate(seq):
            got = trk.update(R.Dets(x, c, k))
            _compare(got, ref.update(R.Dets(x, c, k)), f"round {rnd} frame {f + 1}")
        trk.reset()
        ref.reset()


@pytest.mark.gpu
def test_botsort_rejects_reid_and_unbuilt_gmc_methods():
    """with_reid and the cv2-internal GMC methods (orb / sift / ecc) raise; the default
    sparseOptFlow GMC falls back to the identity warp (with a RuntimeWarning) for frames below its
    64 px minimum or of odd size, like the reference's identity fallbacks (gmc.py:155-158)."""
    BT = _bt()
    with pytest.raises(NotImplementedError):
        BT.BOTSORT(dict(BT.BOTSORT_DEFAULTS, with_reid=True))
    for m in ("orb", "sift", "ecc"):
        with pytest.raises(NotImplementedError):
            BT.BOTSORT(dict(BT.BOTSORT_DEFAULTS, gmc_method=m))
    trk = BT.BOTSORT(dict(BT.BOTSORT_DEFAULTS))
    x, c, k = scenario(3, n_targets=4, n_frames=1)[0]
    with pytest.warns(RuntimeWarning, match="identity warp"):
        out = trk.update(R.Dets(x, c, k), img=np.zeros((8, 8, 3), np.uint8))
    assert out.shape[1] == 8
    assert trk.update(R.Dets(x, c, k)).shape[1] == 8
