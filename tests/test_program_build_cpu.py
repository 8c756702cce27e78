"""yk_program_build (csrc/program.cpp: parse_model rules + Conv/BN fold + lowering + weight
packing in C++, the C-ABI model load of SURVEY 8(b)) against model.py Program on the same state
dict: every yk_op, buffer size, descriptor field and blob byte is identical.  Host-only: the
library is loaded but no device call is made."""
import ctypes as C

import numpy as np
import pytest

from conftest import pkg


def _build_c(L, sd, scale, dtype, fh, fw, imgsz, max_batch):
    w, keep = L.weights_struct(sd)
    h = C.c_void_p()
    L.check(L.lib().yk_program_build(C.byref(w), scale.encode(), dtype, fh, fw, imgsz, max_batch, 300, C.byref(h)),
            "yk_program_build")
    try:
        dp, bp, nb = C.c_void_p(), C.c_void_p(), C.c_int64()
        L.check(L.lib().yk_program_get(h, C.byref(dp), C.byref(bp), C.byref(nb)), "yk_program_get")
        return dp, bp, nb.value, h, keep
    except Exception:
        L.lib().yk_program_destroy(h)
        raise


@pytest.mark.parametrize("scale,dtype,hw,imgsz", [("s", "fp32", (512, 640), 640), ("n", "fp32", (512, 640), 640),
                                                  ("s", "bf16", (500, 640), 640), ("s", "fp8", (1024, 1280), 1280),
                                                  ("n", "bf16", (480, 720), 640), ("s", "fp32", (1024, 1280), 640),
                                                  ("s", "fp16", (512, 640), 640)])
def test_program_build_matches_python_program(scale, dtype, hw, imgsz):
    P = pkg()
    import importlib
    M = importlib.import_module(P.__name__ + ".model")
    L = importlib.import_module(P.__name__ + "._lib")
    ar = P.arch.parse_arch(P.arch.load_model_dict(f"yolov8{scale}-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 3)
    prog = M.Program(ar, sd, hw[0], hw[1], imgsz, 4, dtype)
    want = prog.desc()
    dp, bp, nb, h, keep = _build_c(L, sd, scale, M.ACT[dtype], hw[0], hw[1], imgsz, 4)
    try:
        got = M.ModelDesc.from_address(dp.value)
        for name, _ in M.ModelDesc._fields_:
            if name in ("buf_elems", "ops"):
                continue
            assert getattr(got, name) == getattr(want, name), name
        assert [got.buf_elems[i] for i in range(got.n_bufs)] == prog.buf_elems
        for i in range(got.n_ops):
            assert bytes(got.ops[i]) == bytes(prog.ops[i]), f"op {i}"
        blob = C.string_at(bp.value, nb)
        assert nb == len(prog.blob)
        if blob != bytes(prog.blob):
            a, b = np.frombuffer(blob, np.uint8), np.frombuffer(bytes(prog.blob), np.uint8)
            first = int(np.nonzero(a != b)[0][0])
            pytest.fail(f"blob differs from byte {first} ({int((a != b).sum())} bytes)")
    finally:
        L.lib().yk_program_destroy(h)


def test_program_build_errors():
    P = pkg()
    import importlib
    L = importlib.import_module(P.__name__ + "._lib")
    ar = P.arch.parse_arch(P.arch.load_model_dict("yolov8s-small.yaml"))
    sd = P.weights.synthetic_state_dict(ar, 3)
    h = C.c_void_p()
    w, keep = L.weights_struct(sd)
    assert L.lib().yk_program_build(C.byref(w), b"q", 1, 512, 640, 640, 1, 300, C.byref(h)) != 0
    assert b"scale" in L.lib().yk_last_error()
    assert L.lib().yk_program_build(C.byref(w), b"n", 1, 512, 640, 640, 1, 300, C.byref(h)) != 0  # s weights, n shapes
    assert b"shape" in L.lib().yk_last_error()
    sd2 = {k: v for k, v in sd.items() if k != "model.4.m.1.cv2.bn.running_var"}
    w2, keep2 = L.weights_struct(sd2)
    assert L.lib().yk_program_build(C.byref(w2), b"s", 1, 512, 640, 640, 1, 300, C.byref(h)) != 0
    assert b"model.4.m.1.cv2.bn.running_var" in L.lib().yk_last_error()
