"""The C-ABI model load on the GPU: the detector the library builds itself from a
raw fp32 state dict -- yk_model_load_weights, in-process and from examples/c_host (a C program
reading the raw weights file, no Python step) -- detects exactly what model.py Program's detector
detects: counts and every detection row bit-identical (the programs are byte-identical,
tests/test_program_build_cpu.py, and run the same heuristic kernel plan)."""
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import REPO, pkg

pytestmark = pytest.mark.gpu


def _program_dets(P, ar, sd, frames, dtype, imgsz=640):
    import importlib
    M = importlib.import_module(P.__name__ + ".model")
    H, W = frames[0].shape[:2]
    dm = M.DeviceModel(M.Program(ar, sd, H, W, imgsz, len(frames), dtype))
    d, c = dm.detect(torch.from_numpy(np.stack(frames)).cuda())
    torch.cuda.synchronize()
    return d.cpu().numpy(), c.cpu().numpy()


@pytest.mark.parametrize("scale,dtype", [("s", "fp32"), ("n", "bf16")])
def test_model_load_weights_bit_identical_to_program(scale, dtype):
    import importlib
    P = pkg()
    M = importlib.import_module(P.__name__ + ".model")
    ar = P.arch.parse_arch(P.arch.load_model_dict(f"yolov8{scale}-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 5)
    sc = P.synth.Scene(seed=6, n_targets=24, n_frames=3)
    frames = [sc.frame(t) for t in range(2)]
    want_d, want_c = _program_dets(P, ar, sd, frames, dtype)
    em = M.EngineModel.from_state_dict(sd, scale, dtype, 512, 640, 640, 2)
    d, c = em.detect(torch.from_numpy(np.stack(frames)).cuda())
    torch.cuda.synchronize()
    d, c = d.cpu().numpy(), c.cpu().numpy()
    np.testing.assert_array_equal(c, want_c)
    assert c.sum() > 0
    for b in range(2):
        np.testing.assert_array_equal(d[b, :c[b]], want_d[b, :want_c[b]])


def test_c_host_program_from_raw_state_dict(tmp_path):
    exe = os.path.join(REPO, "examples", "c_host")
    if not os.path.exists(exe):
        pytest.skip("examples/c_host not built (__graft_entry__.build)")
    P = pkg()
    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 7)
    wpath, fpath, opath = tmp_path / "s.ykw", tmp_path / "frames.u8", tmp_path / "out.bin"
    P.weights.save_raw(str(wpath), sd)
    sc = P.synth.Scene(seed=8, n_targets=30, n_frames=3)
    frames = [sc.frame(t) for t in range(2)]
    np.stack(frames).astype(np.uint8).tofile(fpath)
    r = subprocess.run([exe, str(wpath), "s", "1", "512", "640", "640", str(fpath), "2", str(opath)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    raw = opath.read_bytes()
    counts = np.frombuffer(raw, np.int32, 2)
    dets = np.frombuffer(raw, np.float32, 2 * 300 * 6, 8).reshape(2, 300, 6)
    want_d, want_c = _program_dets(P, ar, sd, frames, "fp32")
    np.testing.assert_array_equal(counts, want_c)
    assert counts.sum() > 0
    for b in range(2):
        np.testing.assert_array_equal(dets[b, :counts[b]], want_d[b, :want_c[b]])
