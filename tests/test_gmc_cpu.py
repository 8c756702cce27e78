"""The GMC restatement (oracle/gmc_ref.py: BoT-SORT's sparseOptFlow, ultralytics/trackers/utils/
gmc.py:278-345 with cv2.estimateAffinePartial2D) on the CPU: the RANSAC + Levenberg-Marquardt
estimate recovers a planted similarity through outliers, RANSACUpdateNumIters' limits, and the
whole GMC on a panning camera sequence returns the camera's translation.  cv2 is absent, so these
pin the restatement's behaviour, not cv2's bits (parity with cv2 is unpinned)."""
import numpy as np
import pytest

from gmd_helpers import camera_sequence
from oracle import gmc_ref as R


def test_ransac_lm_recovers_planted_similarity_through_outliers():
    rng = np.random.default_rng(0)
    src = rng.uniform(0, 300, (400, 2)).astype(np.float32)
    a, b, tx, ty = 0.99, 0.02, 3.5, -1.25
    dst = np.stack([a * src[:, 0] - b * src[:, 1] + tx, b * src[:, 0] + a * src[:, 1] + ty], 1).astype(np.float32)
    dst[:40] += rng.uniform(20, 50, (40, 2)).astype(np.float32)  # gross outliers
    dst[40:] += rng.normal(0, 0.2, (360, 2)).astype(np.float32)
    M, mask = R.estimate_affine_partial_2d(src, dst)
    assert mask[:40].sum() == 0 and mask[40:].sum() >= 355
    np.testing.assert_allclose(M, [[a, -b, tx], [b, a, ty]], atol=0.05)
    # the refinement lowers the inliers' squared error below the RANSAC model's
    M0, mask0, it = R.ransac_partial_affine(src, dst)
    inl = mask0.astype(bool)

    def err(m):
        p = src[inl] @ m[:, :2].T + m[:, 2]
        return float(((p - dst[inl]) ** 2).sum())
    assert err(M) <= err(M0) and it >= 1


def test_update_num_iters_limits():
    assert R.update_num_iters(0.99, 0.0, 2, 2000) == 0          # every point an inlier: stop
    assert R.update_num_iters(0.99, 1.0, 2, 2000) == 2000       # no inlier: keep the budget
    n = R.update_num_iters(0.99, 0.5, 2, 2000)                  # log(0.01) / log(0.75)
    assert n == int(np.rint(np.log(0.01) / np.log(0.75)))


def test_cv_rng_is_multiply_with_carry():
    r = R.CvRng()
    s = (1 << 64) - 1
    for _ in range(5):
        s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
        assert r.next() == s & 0xFFFFFFFF
    assert all(0 <= R.CvRng(7).uniform(0, 13) < 13 for _ in range(3))


def test_lane_sum_order():
    v = np.random.default_rng(1).normal(0, 1e8, 1000)
    p = np.zeros(256)
    for k in range(0, 1000, 256):
        c = v[k:k + 256]
        p[: len(c)] += c
    while len(p) > 1:
        p = p[: len(p) // 2] + p[len(p) // 2:]
    assert R.lane_sum(v) == p[0]


@pytest.mark.parametrize("seed", [0, 3])
def test_gmc_on_panning_camera_returns_the_translation(seed):
    """RefGMC('sparseOptFlow') frame by frame: the first frame is the identity; afterwards the
    warp maps the previous frame's points onto the current ones, i.e. its translation is minus the
    camera's offset change (steady pans, 640x512 frames, downscale 2)."""
    frames, off = camera_sequence(seed, 14, h=512, w=640, whip_at=())
    g = R.RefGMC()
    H0 = g.apply(frames[0])
    np.testing.assert_array_equal(H0, np.eye(2, 3))
    for f in range(1, len(frames)):
        H = g.apply(frames[f])
        d = off[f] - off[f - 1]  # (dy, dx)
        assert abs(H[0, 0] - 1) < 0.02 and abs(H[1, 0]) < 0.02, (f, H)
        np.testing.assert_allclose(H[:, 2], [-d[1], -d[0]], atol=1.0, err_msg=f"frame {f}")
        assert g.last["n_points"] > 100 and int(g.last["inliers"].sum()) > 50
