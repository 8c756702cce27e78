"""The CPU oracle reproduces the committed golden fixtures (tests/golden/*.npz, written by
tests/golden/make_golden.py): a regression pin on the oracle itself.  Inputs are regenerated
from seeds; see make_golden.py for what each fixture holds."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402


@pytest.mark.parametrize("name", ["tracker_c3", "tracker_c5", "tracker_defaults", "cmc_jumpy"])
def test_oracle_trackers_reproduce_golden(name):
    want = G.load(name)
    got = G.GENERATORS[name]()
    np.testing.assert_array_equal(got["off"], want["off"])
    np.testing.assert_array_equal(got["ints"], want["ints"])
    np.testing.assert_array_equal(got["stats"], want["stats"])
    np.testing.assert_allclose(got["flts"], want["flts"], rtol=1e-12, atol=1e-12)


def test_oracle_detector_reproduces_golden():
    want = G.load("detector_n")
    got = G.run_detector_oracle()
    np.testing.assert_array_equal(got["n"], want["n"])
    np.testing.assert_allclose(got["dets"], want["dets"], rtol=1e-5, atol=1e-4)
    for b in range(len(want["n"])):
        np.testing.assert_array_equal(got[f"cand_idx{b}"], want[f"cand_idx{b}"])
        np.testing.assert_allclose(got[f"cand{b}"], want[f"cand{b}"], rtol=1e-5, atol=1e-4)


def test_oracle_nms_and_letterbox_reproduce_golden():
    want, got = G.load("nms"), G.run_nms_oracle()
    for k in want:
        np.testing.assert_array_equal(got[k], want[k])
    assert want[f"keep{len(want) - 1}"].tolist() == [0, 1, 2]  # quirk C KAT
    want, got = G.load("letterbox"), G.run_letterbox_oracle()
    for k in want:
        np.testing.assert_array_equal(got[k], want[k])


def test_oracle_global_motion_and_bytetrack_reproduce_golden():
    want, got = G.load("gmd_pan"), G.run_gmd_oracle()
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    assert int(want["stats"][2]) >= 1  # the whip pans reach the reset branch
    want, got = G.load("bytetrack"), G.run_bytetrack_oracle()
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
