"""yk_model_load (engine file written by Program.export_engine) creates the same model the
Python host builds: detections bit-identical to DeviceModel on the same frames and plan."""
import importlib

import numpy as np
import pytest
import torch

from conftest import pkg


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_engine_model_matches_device_model(tmp_path, dtype):
    P = pkg()
    A = importlib.import_module(P.__name__ + ".arch")
    M = importlib.import_module(P.__name__ + ".model")
    W = importlib.import_module(P.__name__ + ".weights")
    ar = A.parse_arch(A.load_model_dict("yolov8n-small.yaml"))
    B = 2
    prog = M.Program(ar, W.synthetic_state_dict(ar, 3), 256, 320, 320, B, dtype)
    plan = [[-1, 0, 0] if o.kind != M.YK_K_CONV else [3, 2, 2] for o in prog.ops]
    path = str(tmp_path / f"n_{dtype}.ykengine")
    prog.export_engine(path, plan, B)
    ref = M.DeviceModel(prog)
    ref.load_plan(B, plan)
    eng = M.EngineModel(path)
    sc = P.synth.Scene(seed=1, n_targets=10, n_frames=4, width=320, height=256)
    frames = sc.frames_torch(0, B, "cuda").contiguous()
    d0, c0 = ref.detect(frames)
    d1, c1 = eng.detect(frames)
    torch.cuda.synchronize()
    c0, c1 = c0.cpu().numpy(), c1.cpu().numpy()
    assert (c0 == c1).all() and c0.sum() > 0
    for b in range(B):
        np.testing.assert_array_equal(d0[b, : c0[b]].cpu().numpy(), d1[b, : c1[b]].cpu().numpy())


@pytest.mark.gpu
def test_engine_rejects_garbage(tmp_path):
    P = pkg()
    M = importlib.import_module(P.__name__ + ".model")
    L = importlib.import_module(P.__name__ + "._lib")
    bad = tmp_path / "bad.ykengine"
    bad.write_bytes(b"NOTANENGINE" + b"\0" * 64)
    with pytest.raises(L.YKError, match="YKENGINE"):
        M.EngineModel(str(bad))
