"""BoT-SORT's global motion compensation on the device (csrc/gmd.hip yk_gmc_apply: gray + 1/2 area
downscale, goodFeaturesToTrack(1000, 0.01, 1, blockSize 3), pyramidal LK, RANSAC + Levenberg-
Marquardt estimateAffinePartial2D; csrc/bytetrack.hip yk_bt_step_warp: multi_gmc and the dense-
covariance Kalman steps) against oracle/gmc_ref.py + oracle/bytetrack_ref.py on panning camera
sequences.

Bars: corners, LK end points and status bit-identical to the restatement; the RANSAC point /
inlier / iteration counts identical; the warp within 1e-9 (the same operations in the same order;
libm log / sqrt may differ in the last ulp).  BoT-SORT with GMC: the same rows, ids, scores and
classes every frame, boxes within 1e-3 px (numpy's BLAS sums the dense covariance products in its
own order).  Parity with cv2 itself is unpinned (cv2 is absent)."""
import numpy as np
import pytest

from conftest import pkg
from gmd_helpers import camera_sequence
from oracle import bytetrack_ref as BR
from oracle import gmc_ref as R

pytestmark = pytest.mark.gpu


def _gmc(P):
    import importlib

    return importlib.import_module(P.__name__ + ".bytetrack").GMC()


@pytest.mark.parametrize("seed,whip", [(0, ()), (5, (7,))])
def test_device_gmc_matches_restatement(seed, whip):
    P = pkg()
    frames, off = camera_sequence(seed, 16, h=512, w=640, whip_at=whip)
    dev, ref = _gmc(P), R.RefGMC()
    states = []
    for f, fr in enumerate(frames):
        kp_prev = None if ref.prevKeyPoints is None else ref.prevKeyPoints.reshape(-1, 2).copy()
        H = dev.apply(fr)
        Hr = ref.apply(fr)
        info = dev.info()[0]
        states.append(int(info[4]))
        if f == 0:
            np.testing.assert_array_equal(H, np.eye(2, 3))
            continue
        c, nx, st = dev.points(0)  # the previous frame's keypoints, tracked into this frame
        np.testing.assert_array_equal(c, kp_prev, err_msg=f"frame {f}: corners")
        np.testing.assert_array_equal(st, ref.last["status"], err_msg=f"frame {f}: LK status")
        ok = st.astype(bool)
        np.testing.assert_array_equal(nx[ok], ref.last["next"].reshape(-1, 2)[ok], err_msg=f"frame {f}: LK points")
        assert int(info[0]) == ref.last["n_points"], (f, info, ref.last["n_points"])
        assert int(info[1]) == int(ref.last["inliers"].sum()), (f, info)
        np.testing.assert_allclose(H, Hr, rtol=1e-9, atol=1e-9, err_msg=f"frame {f}: warp")
    print("GMC_STATES", seed, states)
    assert states[0] == 0 and all(s == 1 for s in states[1:])


def _pan_detections(off, n=14, seed=0, h=512, w=640):
    """Boxes fixed in the world, seen through the panning camera (they move with the pan), with
    jitter and a few dropouts: float32 rows [x1 y1 x2 y2 conf cls] per frame."""
    rng = np.random.default_rng(seed)
    anc = np.stack([rng.uniform(80, w - 120, n), rng.uniform(80, h - 120, n)], 1) + off[0][::-1]
    size = rng.uniform(18, 40, (n, 2))
    out = []
    for f in range(len(off)):
        cx = anc[:, 0] - off[f, 1] + rng.normal(0, 0.4, n)
        cy = anc[:, 1] - off[f, 0] + rng.normal(0, 0.4, n)
        keep = (rng.random(n) > 0.08) & (cx > 10) & (cx < w - 10) & (cy > 10) & (cy < h - 10)
        sc = rng.uniform(0.3, 0.95, n)
        rows = np.stack([cx - size[:, 0] / 2, cy - size[:, 1] / 2, cx + size[:, 0] / 2, cy + size[:, 1] / 2, sc,
                         np.zeros(n)], 1)[keep]
        out.append(rows.astype(np.float32))
    return out


@pytest.mark.parametrize("method", ["sparseOptFlow", "none"])
def test_botsort_with_gmc_matches_oracle(method):
    """BOTSORT(botsort.yaml defaults, gmc_method) stepped with the frame, device vs oracle, on a
    slow-then-fast panning sequence whose targets move with the camera."""
    import importlib

    P = pkg()
    BT = importlib.import_module(P.__name__ + ".bytetrack")
    frames, off = camera_sequence(2, 40, h=512, w=640, whip_at=())
    dets = _pan_detections(off)
    cfg = dict(BR.BOTSORT_CFG, gmc_method=method)
    dev = BT.BOTSORT(cfg)
    ref = BR.RefTracker(cfg, ids=BR.IdCounter())
    n_rows, maxdev = 0, 0.0
    for f in range(len(frames)):
        d = dets[f]
        got = dev.update(d, frames[f])
        want = ref.update(BR.Dets(d[:, :4], d[:, 4], d[:, 5]), frames[f]).reshape(-1, 8)
        assert got.shape == want.shape, (f, got.shape, want.shape)
        np.testing.assert_array_equal(got[:, 4:], want[:, 4:], err_msg=f"frame {f}: id / score / cls / idx")
        if len(want):
            dv = float(np.max(np.abs(got[:, :4] - want[:, :4])))
            maxdev = max(maxdev, dv)
            assert dv <= 1e-3, (f, got[:, :4], want[:, :4])
        n_rows += len(want)
    print("BOTSORT_GMC", method, {"rows": n_rows, "max_box_dev_px": maxdev})
    # without compensation the fast pan loses its tracks (that is what GMC is for): fewer rows
    assert n_rows > (200 if method == "sparseOptFlow" else 100)


def test_gmc_reset_params_then_apply():
    """GMC.reset_params() (gmc.py:347-353) mid-sequence: the next apply is a first frame again (the
    identity, every wave of gmc_kernel on the same branch -- ADVICE r4: has_prev was read by every
    thread while thread 0 set it), and the frames after it match a fresh restatement fed from the
    reset on."""
    P = pkg()
    frames, _ = camera_sequence(3, 12, h=512, w=640, whip_at=(8,))
    dev = _gmc(P)
    for fr in frames[:5]:
        dev.apply(fr)
    dev.reset_params()
    ref = R.RefGMC()
    for f, fr in enumerate(frames[5:]):
        H = dev.apply(fr)
        Hr = ref.apply(fr)
        if f == 0:
            np.testing.assert_array_equal(H, np.eye(2, 3))
            assert int(dev.info()[0][4]) == 0
            continue
        assert int(dev.info()[0][4]) == 1, (f, dev.info())
        np.testing.assert_allclose(H, Hr, rtol=1e-9, atol=1e-9, err_msg=f"frame {f} after reset: warp")


def test_gmc_odd_frame_size_falls_back_to_identity():
    """An odd frame (1242x375, KITTI-like) is outside the restated exact-1/2 downscale: GMC returns
    the identity with one RuntimeWarning instead of failing, every frame."""
    P = pkg()
    dev = _gmc(P)
    rng = np.random.default_rng(0)
    fr = rng.integers(0, 255, (375, 1242, 3), dtype=np.uint8)
    with pytest.warns(RuntimeWarning, match="not even"):
        H = dev.apply(fr)
    np.testing.assert_array_equal(H, np.eye(2, 3))
    np.testing.assert_array_equal(dev.apply(np.roll(fr, 3, axis=1)), np.eye(2, 3))
