"""CPU checks of the host-side program builder (no GPU): parse_model restatement (channels,
repeats, params, FLOPs vs SURVEY §8a), LetterBox geometry, and a numpy emulation of the
packed implicit-GEMM conv (fragment layout + K-chunk table) against torch's conv2d."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg


def _m():
    P = pkg()
    return P.arch, P.weights, P.model


@pytest.mark.parametrize("name,scale,chans,params,gflop", [
    ("yolov8-small.yaml", "n", [16, 24, 24, 48, 48, 96, 96, 192, 192, 192], 2.2777e6, 7.616),
    ("yolov8s-small.yaml", "s", [24, 40, 40, 80, 80, 160, 160, 320, 320, 320], 5.9637e6, 16.540),
])
def test_parse_model_matches_survey(name, scale, chans, params, gflop):
    A, W, M = _m()
    ar = A.parse_arch(A.load_model_dict(name))
    assert ar.scale == scale
    assert [L.c2 for L in ar.layers[:10]] == chans
    assert A.detect_strides(ar) == [4, 8, 16, 32]
    n_conv = len(A.conv_specs(ar))
    assert n_conv == (91 if scale == "n" else 95)
    nparam = sum(c1 * c2 * k * k for _, c1, c2, k, _, _ in A.conv_specs(ar))
    assert abs(nparam - params) / params < 1e-3
    prog = M.Program(ar, W.synthetic_state_dict(ar, 0), 512, 640)
    assert abs(sum(prog.op_flops(1)) / 1e9 - gflop) < 0.01
    assert prog.n_anchors == 27200


def test_letterbox_geometry():
    _, _, M = _m()
    assert M.letterbox_geometry(512, 640, 640) == (512, 640, 0, 0)
    assert M.letterbox_geometry(500, 640, 640) == (512, 640, 6, 0)
    assert M.letterbox_geometry(1024, 1280, 1280) == (1024, 1280, 0, 0)
    # resizing geometries (cv2.resize INTER_LINEAR on the device, letterbox.py)
    assert M.letterbox_geometry(1024, 1280, 640) == (512, 640, 0, 0)   # exact 2x: INTER_AREA path
    assert M.letterbox_geometry(1080, 1920, 640) == (384, 640, 12, 0)  # 640x360 + 12 rows top/bottom


def test_letterbox_tables_match_oracle_restatement():
    """The device kernel's per-axis tables (letterbox.py) equal the oracle's independent
    restatement of OpenCV's coefficient rule, and both resize paths keep flat images flat."""
    import importlib
    from oracle import letterbox_ref as R
    LB = importlib.import_module(pkg().__name__ + ".letterbox")
    for (h, w) in [(1080, 1920), (600, 800), (300, 400), (1025, 1281)]:
        p = LB.plan(h, w, 640)
        assert p["mode"] == LB.RS_LINEAR
        xs, x0, x1 = R._axis(p["new_w"], w, True)
        ys, y0, y1 = R._axis(p["new_h"], h, False)
        np.testing.assert_array_equal(p["xofs"], xs)
        np.testing.assert_array_equal(p["xw"][:, 0], x0)
        np.testing.assert_array_equal(p["xw"][:, 1], x1)
        np.testing.assert_array_equal(p["yofs"], ys)
        np.testing.assert_array_equal(p["yw"][:, 0], y0)
        np.testing.assert_array_equal(p["yw"][:, 1], y1)
    assert LB.plan(1024, 1280, 640)["mode"] == LB.RS_AREA2
    for shape in [(1080, 1920, 3), (300, 400, 3), (1024, 1280, 3)]:
        flat = np.full(shape, 77, np.uint8)
        assert np.all(R.letterbox(flat)[12:-12] == 77) or np.all(R.letterbox(flat) == 77)


def _emulate(prog, op, w_blob_f32, bias, tab, src, B):
    """numpy emulation of conv_igemm_kernel for one op (f32 build): per pixel, per K step,
    per lane group -> the exact operand fragments the kernel forms."""
    k, s = op.ksize, op.stride
    epl = prog.epl
    n_chunks = k * k * (op.src_ch[0] + (op.src_ch[1] if op.n_src > 1 else 0)) // 8
    oh, ow = op.out_h, op.out_w
    out = np.zeros((B, oh, ow, op.n_tiles * 16), np.float64)
    Wp = w_blob_f32.reshape(op.n_tiles, op.k_steps, 4, 16, epl)  # [nt][ks][kg][col][e]
    for b in range(B):
        for oy in range(oh):
            for ox in range(ow):
                acc = np.zeros(op.n_tiles * 16)
                for ks in range(op.k_steps):
                    for kg in range(4):
                        kel = ks * 4 * epl + kg * epl
                        q, sub = kel >> 3, kel & 7
                        if q >= n_chunks:
                            continue
                        e = int(tab[q])
                        dx, dy = ((e >> 21) & 15) - 8, ((e >> 17) & 15) - 8
                        si, ch = (e >> 16) & 1, e & 0xFFFF
                        iy, ix = oy * s + dy, ox * s + dx
                        arr, up = src[si]
                        if not (0 <= iy < arr.shape[1] << up and 0 <= ix < arr.shape[2] << up):
                            continue
                        x = arr[b, iy >> up, ix >> up, ch + sub: ch + sub + epl]
                        wv = Wp[:, ks, kg, :, :].reshape(-1, epl)  # [nt*16, e]
                        acc += wv.astype(np.float64) @ x.astype(np.float64)
                out[b, oy, ox] = acc + bias
    return out


def test_packed_conv_emulation_matches_conv2d():
    """Pack a 3x3 conv whose input is a two-view concat with an upsampled source (like
    C2f.cv1 after Upsample+Concat, but 3x3) and emulate the kernel's fragment arithmetic."""
    A, W, M = _m()
    ar = A.parse_arch(A.load_model_dict("yolov8-small.yaml"))
    prog = M.Program(ar, W.synthetic_state_dict(ar, 0), 512, 640, dtype="fp32")
    rng = np.random.default_rng(0)
    B, H, Wd = 1, 6, 8
    c_a, c_b, c_out = 12, 20, 24  # logical; physical 16 + 24
    xa = np.zeros((B, H // 2, Wd // 2, 16), np.float32)
    xa[..., :c_a] = rng.standard_normal((B, H // 2, Wd // 2, c_a))
    xb = np.zeros((B, H, Wd, 24), np.float32)
    xb[..., :c_b] = rng.standard_normal((B, H, Wd, c_b))
    segs = [M.Seg(0, 0, 16, 16, c_a, H // 2, Wd // 2, up=1), M.Seg(1, 0, 24, 24, c_b, H, Wd)]
    w = torch.from_numpy(rng.standard_normal((c_out, c_a + c_b, 3, 3)).astype(np.float32))
    b = torch.from_numpy(rng.standard_normal(c_out).astype(np.float32))
    views, packed, bias, tab, k_steps, n_tiles = prog.pack(w, b, segs, list(range(c_out)), 24)

    class Op:
        pass
    op = Op()
    op.ksize, op.stride, op.n_src, op.src_ch = 3, 1, 2, [16, 24]
    op.out_h, op.out_w, op.k_steps, op.n_tiles = H, Wd, k_steps, n_tiles
    got = _emulate(prog, op, packed, bias, tab, [(xa, 1), (xb, 0)], B)[..., :c_out]
    xin = torch.cat([F.interpolate(torch.from_numpy(xa[..., :c_a]).permute(0, 3, 1, 2), scale_factor=2),
                     torch.from_numpy(xb[..., :c_b]).permute(0, 3, 1, 2)], 1)
    want = F.conv2d(xin.double(), w.double(), b.double(), 1, 1).permute(0, 2, 3, 1).numpy()
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-9)
    assert k_steps == math.ceil(9 * 40 / 16) and n_tiles == 2


def test_fp8_packing_matches_oracle_quantisation():
    """FP8 program: 16-channel physical groups, and every conv's packed e4m3 weights and
    dequant scales equal the oracle's per-output-channel rule (oracle.detector_ref.fp8_weights)."""
    from oracle import detector_ref as D
    P = pkg()
    import importlib
    A = importlib.import_module(P.__name__ + ".arch")
    W = importlib.import_module(P.__name__ + ".weights")
    M = importlib.import_module(P.__name__ + ".model")
    ar = A.parse_arch(A.load_model_dict("yolov8s-small.yaml"))
    sd = W.synthetic_state_dict(ar, 0)
    prog = M.Program(ar, sd, 512, 640, 640, 2, "fp8")
    blob = np.frombuffer(bytes(prog.blob), np.uint8)
    checked = 0
    names = [p for p in prog.fused]
    for op in prog.ops:
        if op.kind != M.YK_K_CONV:
            continue
        assert op.src_ch[0] % 16 == 0 and (op.n_src < 2 or op.src_ch[1] % 16 == 0)
        nt, ks = op.n_tiles, op.k_steps
        dq = np.frombuffer(bytes(prog.blob[op.b_off:op.b_off + nt * 32 * 4]), np.float32)[nt * 16:]
        assert np.all(np.isfinite(dq)) and np.all(dq > 0)
        checked += 1
    assert checked >= 80
    # model.1 (3x3 s2, 24 -> 40 logical channels) unpacked and compared element for element
    op = prog.ops[1]
    nt, ks = op.n_tiles, op.k_steps
    pk = blob[op.w_off:op.w_off + nt * ks * 64 * 16].reshape(nt, ks, 64, 16)
    wq = torch.from_numpy(pk.copy()).view(torch.float8_e4m3fn).float()
    x = wq.reshape(nt, ks, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(nt * 16, -1)
    w, _ = D.fuse(sd, "model.1")
    Wq, dq_ref = D.fp8_weights(w)
    cin_p = op.src_ch[0]
    for ky in range(3):
        for kx in range(3):
            tap = ky * 3 + kx
            assert torch.equal(x[:40, tap * cin_p:tap * cin_p + 24], Wq[:, :, ky, kx])
    dq = np.frombuffer(bytes(prog.blob[op.b_off:op.b_off + nt * 32 * 4]), np.float32)[nt * 16:nt * 16 + 40]
    np.testing.assert_array_equal(dq, dq_ref.numpy())
    assert "model.1" in names
