"""§8f-2: an ultralytics-style best.pt (pickled DetectionModel, fp16, YAML on model.yaml) is read
with torch.load(weights_only=True) and inert stand-ins for its classes, into the reference's
state-dict naming and model YAML (nn/tasks.py:1404-1521, utils/torch_utils.py:714-773).  The
reference ships no best.pt, so the fixture is written by tests/ckpt_helpers.py."""
import numpy as np
import pytest
import torch

from conftest import pkg
from ckpt_helpers import write_checkpoint


@pytest.fixture(scope="module")
def fake_ckpt(tmp_path_factory):
    P = pkg()
    y = P.arch.load_model_dict("yolov8-small.yaml")  # the trained run's model (scale n)
    ar = P.arch.parse_arch(y)
    sd = P.weights.synthetic_state_dict(ar, 3)
    path = str(tmp_path_factory.mktemp("ckpt") / "best.pt")
    write_checkpoint(path, ar, y, sd, half=True)
    return path, y, ar, sd


def test_checkpoint_roundtrip_state_dict_and_yaml(fake_ckpt):
    import importlib

    path, y, ar, sd = fake_ckpt
    CK = importlib.import_module(pkg().__name__ + ".checkpoint")
    ydict, got, meta = CK.load_checkpoint(path)
    assert ydict["backbone"] == y["backbone"]
    assert set(got) == set(sd)
    for k, v in sd.items():
        want = v.half().float() if v.is_floating_point() else v
        assert got[k].dtype == want.dtype, k
        assert torch.equal(got[k], want), k
    assert meta["version"] == "8.3.193" and meta["epoch"] == -1
    P = pkg()
    ar2 = P.arch.parse_arch(ydict)
    assert ar2.scale == "n"  # yolov8-small.yaml names no scale: parse_model takes the first (n)
    assert [(L.kind, L.c2) for L in ar2.layers] == [(L.kind, L.c2) for L in ar.layers]


def test_checkpoint_load_runs_nothing_from_the_file(fake_ckpt, tmp_path):
    """A pickle that REDUCEs os.system is stubbed, not executed."""
    import importlib
    import pickle

    class Evil:
        def __reduce__(self):
            import os
            return (os.system, ("touch " + str(tmp_path / "pwned"),))

    p = tmp_path / "evil.pt"
    with open(p, "wb") as f:
        pickle.dump({"model": Evil()}, f)
    CK = importlib.import_module(pkg().__name__ + ".checkpoint")
    with pytest.raises(Exception):
        CK.load_checkpoint(str(p))
    assert not (tmp_path / "pwned").exists()
