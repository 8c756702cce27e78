"""The reference driver example (examples/aircraft_detection_tracking.py) end to end on the GPU:
frame stack in, visualised frame stack out, through the compat imports."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_driver_example_runs(tmp_path):
    P = pkg()
    sc = P.synth.Scene(seed=9, n_targets=10, n_frames=12)
    np.save(tmp_path / "in.npy", np.stack([sc.frame(t) for t in range(12)]))
    r = subprocess.run([sys.executable, os.path.join(REPO, "examples", "aircraft_detection_tracking.py"),
                        "--source", str(tmp_path / "in.npy"), "--out", str(tmp_path / "out.npy"), "--dtype", "fp32"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "frames 12" in r.stdout
    out = np.load(tmp_path / "out.npy")
    assert out.shape == (12, 512, 640, 3) and out.dtype == np.uint8
    assert (out != np.load(tmp_path / "in.npy")).any()
