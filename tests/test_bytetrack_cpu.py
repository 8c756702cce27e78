"""ByteTrack / BoT-SORT checker pieces on the CPU: the CPython set-order restatement the device
reproduces, the oracle's block-filter identities the device kernel relies on, the ABI mirror."""
import random

import numpy as np
import pytest

from oracle import bytetrack_ref as R
from oracle.pyset_order import frozenset_diff_order

from bt_helpers import scenario


def test_frozenset_order_restatement_matches_cpython():
    rng = random.Random(0)
    nonasc = 0
    for _ in range(4000):
        n = rng.randint(0, 300)
        ex = rng.sample(range(n), rng.randint(0, n))
        ref = [int(v) for v in list(frozenset(np.arange(n)) - frozenset(np.asarray(ex, dtype=np.int64)))]
        assert frozenset_diff_order(n, ex) == ref
        nonasc += ref != sorted(ref)
    assert nonasc > 100  # the order really is not ascending in general


@pytest.mark.parametrize("kind", ["xyah", "xywh"])
def test_block_filter_identities(kind):
    """The device keeps P as four 2x2 blocks; the oracle's 8x8 numpy / scipy calls reduce to the
    block formulas of csrc/bytetrack.hip (predict exactly; update to the OpenBLAS reciprocal
    dtrsm, checked to 1 ulp)."""
    rng = np.random.default_rng(3)
    for t in range(300):
        mean = rng.uniform(1, 300, 8)
        mean[4:] = rng.normal(0, 2, 4)
        P = np.zeros((8, 8))
        for c in range(4):
            P[c, c], P[c, c + 4], P[c + 4, c + 4] = rng.uniform(1, 50), rng.uniform(-5, 5), rng.uniform(1, 20)
            P[c + 4, c] = P[c, c + 4]
        m2, P2 = R.kf_multi_predict(kind, mean[None].copy(), P[None].copy())
        for c in range(4):
            ref = mean[3] if kind == "xyah" else mean[2 + (c & 1)]
            sp = 1e-2 if (kind == "xyah" and c == 2) else R._WP * ref
            sv = 1e-5 if (kind == "xyah" and c == 2) else R._WV * ref
            p, a, b, v = P[c, c], P[c, c + 4], P[c + 4, c], P[c + 4, c + 4]
            assert m2[0, c] == mean[c] + mean[c + 4]
            assert P2[0, c, c] == ((p + b) + (a + v)) + sp * sp
            assert P2[0, c + 4, c + 4] == v + sv * sv
        meas = rng.uniform(1, 300, 4).astype(np.float32)
        mu, Pu = R.kf_update(kind, mean.copy(), P.copy(), meas)
        for c in range(4):
            ref = mean[3] if kind == "xyah" else mean[2 + (c & 1)]
            r = (0.1 if (kind == "xyah" and c == 2) else R._WP * ref) ** 2
            p, b = P[c, c], P[c + 4, c]
            S = p + r
            il = 1.0 / np.sqrt(S)
            kc = (p * il) * il
            np.testing.assert_allclose(mu[c], mean[c] + (float(meas[c]) - mean[c]) * kc, rtol=1e-15, atol=0)


def test_oracle_runs_both_trackers_with_shared_ids():
    ids = R.IdCounter()
    trk = [R.RefTracker(None, ids=ids), R.RefTracker(dict(R.BOTSORT_CFG), ids=ids)]
    ids.reset()
    seqs = [scenario(1, n_targets=12, n_frames=30), scenario(2, n_targets=12, n_frames=30)]
    seen = set()
    for f in range(30):
        for s in range(2):
            xyxy, conf, cls = seqs[s][f]
            out = trk[s].update(R.Dets(xyxy, conf, cls))
            assert out.dtype == np.float32 and (out.size == 0 or out.shape[1] == 8)
            seen.update(out[:, 4].astype(int).tolist() if out.size else [])
    assert len(seen) > 10 and ids.count >= max(seen)



def test_lap_branch_known_answer_differs_from_scipy():
    """matching.linear_assignment's default lap branch (lapjv, extend_cost, cost_limit = thresh)
    against the scipy branch on the case where they part: rows A, B; columns d1, d2; costs
    A-d1 0.4, A-d2 0.85, B-d1 0.5, B-d2 1 (no overlap); thresh 0.8.  scipy assigns A-d2 + B-d1
    (1.35 < 1.4) and its filter keeps only B-d1; lapjv's extended problem keeps A-d1 (0.4 - 0.8
    beats 0.5 - 0.8) and leaves B and d2 unmatched, the lists ascending."""
    cost = np.array([[0.4, 0.85], [0.5, 1.0]], np.float32)
    m, ua, ub = R.linear_assignment(cost, 0.8)
    assert [list(p) for p in m] == [[0, 0]] and list(ua) == [1] and list(ub) == [1]
    m, ua, ub = R.linear_assignment(cost, 0.8, use_lap=False)
    assert [list(p) for p in m] == [[1, 0]] and list(ua) == [0] and list(ub) == [1]
    # the matched set maximises the summed margins thresh - cost: A-d2 alone (0.6) beats A-d1 +
    # B-d2 (0.3 + 0.1), and B-d1 (cost above thresh) is never kept; empty matrices give the
    # tuple(range(...)) lists
    x, y = R.lapjv_extended(np.array([[0.5, 0.2], [0.9, 0.7]]), 0.8)
    assert list(x) == [1, -1] and list(y) == [-1, 0]
    m, ua, ub = R.linear_assignment(np.zeros((0, 3), np.float32), 0.8)
    assert len(m) == 0 and ua == () and ub == (0, 1, 2)
