"""Detector program builder: parsed model + fused weights -> a libyk.so program.

The reference executes the parsed graph module by module (nn/tasks.py:159-188) with
torch.cat / chunk / nn.Upsample materialising every intermediate.  Here the graph is
lowered once, on the host, into a flat op list over NHWC activation buffers that stay
resident in HBM:

  * every logical channel group is padded to a multiple of 8 (16-byte bf16 fragments);
  * Concat and C2f's chunk/cat become channel slices: producers write straight into
    the consumer's buffer, a consumer reads up to two views (K-space concatenation);
  * nn.Upsample(2, nearest) is folded into the consumer's gather (view.up = 1);
  * Detect's two first 3x3 convs share their input and are fused into one conv with
    N = 64 + c3; its final 1x1 convs are fused into the decode kernel.

Weights are packed per conv for the MFMA A operand: [n_tiles][k_steps][64 lanes][16 B],
K ordered (tap, physical input channel), together with an int32 table that maps every
8-channel K chunk to (dy, dx, source view, channel).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, replace

import numpy as np
import torch

from . import _lib as L
from . import arch as A
from . import letterbox as LB
from . import weights as Wt

YK_K_CONV_INPUT, YK_K_CONV, YK_K_SPPF_POOL, YK_K_DETECT = range(4)
ACT = {"bf16": 0, "fp32": 1, "fp8": 2, "fp16": 3}
ESZ = {"bf16": 2, "fp32": 4, "fp8": 1, "fp16": 2}


def phys(c: int, align: int = 8) -> int:
    return (c + align - 1) // align * align


class View(C.Structure):
    _fields_ = [("buf", C.c_int32), ("c_off", C.c_int32), ("c_stride", C.c_int32), ("h", C.c_int32),
                ("w", C.c_int32), ("up", C.c_int32)]


class Op(C.Structure):
    _fields_ = [("kind", C.c_int32), ("ksize", C.c_int32), ("stride", C.c_int32), ("act", C.c_int32),
                ("n_src", C.c_int32), ("src", View * 2), ("src_ch", C.c_int32 * 2), ("dst", View),
                ("cout", C.c_int32), ("has_res", C.c_int32), ("res", View), ("out_h", C.c_int32),
                ("out_w", C.c_int32), ("k_steps", C.c_int32), ("n_tiles", C.c_int32), ("w_off", C.c_int64),
                ("b_off", C.c_int64), ("t_off", C.c_int64), ("det_stride", C.c_int32),
                ("det_anchor_off", C.c_int32), ("det_cls_off", C.c_int32), ("det_cls_ch", C.c_int32),
                ("det_wc_off", C.c_int64)]


class ModelDesc(C.Structure):
    _fields_ = [("act_dtype", C.c_int32), ("max_batch", C.c_int32), ("frame_h", C.c_int32), ("frame_w", C.c_int32),
                ("in_h", C.c_int32), ("in_w", C.c_int32), ("pad_top", C.c_int32), ("pad_left", C.c_int32),
                ("n_anchors", C.c_int32), ("nc", C.c_int32), ("max_det", C.c_int32), ("n_bufs", C.c_int32),
                ("buf_elems", C.POINTER(C.c_int64)), ("n_ops", C.c_int32), ("ops", C.POINTER(Op)),
                ("rs_mode", C.c_int32), ("rs_w", C.c_int32), ("rs_h", C.c_int32), ("box_pad_x", C.c_int32),
                ("box_pad_y", C.c_int32), ("box_gain", C.c_float), ("rs_tab_off", C.c_int64)]


@dataclass(frozen=True)
class Seg:
    """One logical channel group stored in a buffer: cl logical channels at c_off (padded to cp)."""
    buf: int
    c_off: int
    c_stride: int
    cp: int
    cl: int
    h: int      # stored spatial size
    w: int
    up: int = 0  # log2 upsample applied when read

    @property
    def lh(self):  # logical (as read) size
        return self.h << self.up

    @property
    def lw(self):
        return self.w << self.up


def letterbox_geometry(frame_h, frame_w, imgsz=640, stride=32):
    """LetterBox(auto=True, center=True) geometry (data/augment.py:1698-1729).  Returns
    (in_h, in_w, pad_top, pad_left); see letterbox.plan for the resize tables."""
    p = LB.plan(frame_h, frame_w, imgsz, stride)
    return p["in_h"], p["in_w"], p["top"], p["left"]


def _bf16_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> bfloat16 bit patterns, round-to-nearest-even (torch's conversion)."""
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16).view(torch.int16).numpy()


def _f16_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> IEEE binary16 bits, round to nearest even (torch's .half())."""
    return np.ascontiguousarray(a, dtype=np.float32).astype(np.float16).view(np.int16)


def _fp8_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> OCP e4m3 (float8_e4m3fn) bytes, round-to-nearest-even, |a| <= 448."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).clamp(-448.0, 448.0)
    return t.to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def fp8_round(t: torch.Tensor) -> torch.Tensor:
    """Values as stored in an FP8 activation buffer (saturated e4m3, round-to-nearest-even)."""
    return t.float().clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()


class Program:
    def __init__(self, ar: A.Arch, sd: dict, frame_h: int, frame_w: int, imgsz=640, max_batch: int = 8,
                 dtype: str = "bf16", max_det: int = 300):
        if dtype not in ACT:
            raise ValueError(f"dtype must be one of {sorted(ACT)}")
        self.ar, self.dtype, self.max_batch, self.max_det = ar, dtype, int(max_batch), int(max_det)
        self.frame_h, self.frame_w = int(frame_h), int(frame_w)
        self.strides = A.detect_strides(ar)
        self.lb = LB.plan(frame_h, frame_w, imgsz, max(self.strides))
        self.in_h, self.in_w, self.pad_top, self.pad_left = self.lb["in_h"], self.lb["in_w"], self.lb["top"], self.lb["left"]
        self.epl = 16 // ESZ[dtype]  # K elements per lane per 16-byte fragment
        self.fused = Wt.fused_convs(sd, ar)
        self.sd = sd
        self.buf_elems: list[int] = []
        self.ops: list[Op] = []
        self.blob = bytearray()
        self.layer_out: dict[int, list[Seg]] = {}
        self.op_meta: list[int] = []  # MACs per image of each op
        self.n_anchors = 0
        self._build()
        self.rs_tab_off = self.add_blob(LB.table_blob(self.lb))

    def phys(self, c: int) -> int:
        """Physical channels of a logical group: a whole number of 16-byte... K chunks; FP8
        fragments span 16 channels, so a chunk never straddles a tap or a concat source."""
        return phys(c, 16 if self.dtype == "fp8" else 8)

    # -- resources -------------------------------------------------------------
    def new_buf(self, h, w, c) -> int:
        self.buf_elems.append(int(h) * int(w) * int(c))
        return len(self.buf_elems) - 1

    def add_blob(self, arr: np.ndarray) -> int:
        off = (len(self.blob) + 255) // 256 * 256
        self.blob.extend(b"\0" * (off - len(self.blob)))
        self.blob.extend(np.ascontiguousarray(arr).tobytes())
        return off

    # -- packing -----------------------------------------------------------------
    @staticmethod
    def views_of(segs):
        """Merge consecutive contiguous segs of one buffer into <= 2 read views."""
        views = []  # [first seg, cp_total, [(seg, k_offset_within_view)]]
        for s in segs:
            if views:
                v = views[-1]
                f = v[0]
                if s.buf == f.buf and s.up == f.up and s.c_off == f.c_off + v[1] and s.c_stride == f.c_stride:
                    v[2].append((s, v[1]))
                    v[1] += s.cp
                    continue
            views.append([s, s.cp, [(s, 0)]])
        if len(views) > 2:
            raise ValueError("a conv may read at most two views")
        return views

    def pack(self, w: torch.Tensor, b: torch.Tensor, src_segs, out_map, cout_p):
        """W [c2, c1, k, k] (logical) -> packed MFMA operand blob + bias + K-chunk table."""
        w = w.numpy().astype(np.float32)
        b = b.numpy().astype(np.float32)
        c2, c1, k, _ = w.shape
        views = self.views_of(src_segs)
        cin_p = sum(v[1] for v in views)
        in_map = []
        kbase = 0
        for v in views:
            for s, off in v[2]:
                in_map.extend(kbase + off + j for j in range(s.cl))
            kbase += v[1]
        assert len(in_map) == c1, (len(in_map), c1)
        K = k * k * cin_p
        kstep = 4 * self.epl
        k_steps = math.ceil(K / kstep)
        n_tiles = math.ceil(cout_p / 16)
        Wp = np.zeros((n_tiles * 16, k_steps * kstep), np.float32)
        om = np.asarray(out_map)
        im = np.asarray(in_map)
        for ky in range(k):
            for kx in range(k):
                tap = ky * k + kx
                Wp[np.ix_(om, tap * cin_p + im)] = w[:, :, ky, kx]
        if self.dtype == "fp8":
            # per-output-channel scale: the row's max |w| maps to e4m3's 448; the kernel
            # multiplies the accumulator by the inverse (dq) before adding the bias
            amax = np.abs(Wp).max(axis=1)
            scale = np.where(amax > 0, 448.0 / np.maximum(amax, 1e-30), 1.0).astype(np.float32)
            dq = (1.0 / scale).astype(np.float32)
            Wp = Wp * scale[:, None]
        P = Wp.reshape(n_tiles, 16, k_steps, 4, self.epl).transpose(0, 2, 3, 1, 4)  # [nt][ks][kg][col][e]
        P = P.reshape(n_tiles, k_steps, 64, self.epl)
        bias = np.zeros(n_tiles * 16, np.float32)
        bias[om] = b
        if self.dtype == "fp8":
            packed = _fp8_bits(P)
            bias = np.concatenate([bias, dq])
        else:
            packed = _bf16_bits(P) if self.dtype == "bf16" else _f16_bits(P) if self.dtype == "fp16" else P
        tab = []
        pad = k // 2
        for q in range(K // 8):
            tap, ch = divmod(q * 8, cin_p)
            dy, dx = tap // k - pad, tap % k - pad
            src = 0 if ch < views[0][1] else 1
            off = ch if src == 0 else ch - views[0][1]
            tab.append(((dx + 8) << 21) | ((dy + 8) << 17) | (src << 16) | off)
        tab = np.asarray(tab or [-1], np.int32)
        return views, packed, bias, tab, k_steps, n_tiles

    def conv_op(self, prefix, src_segs, dst: Seg, out_map, cout_p, res: Seg | None = None):
        w, b, k, s, act = self.fused[prefix]
        views, packed, bias, tab, k_steps, n_tiles = self.pack(w, b, src_segs, out_map, cout_p)
        op = Op()
        op.kind = YK_K_CONV
        op.ksize, op.stride, op.act = k, s, int(bool(act))
        op.n_src = len(views)
        for i, v in enumerate(views):
            f = v[0]
            op.src[i] = View(f.buf, f.c_off, f.c_stride, f.h, f.w, f.up)
            op.src_ch[i] = v[1]
        op.dst = View(dst.buf, dst.c_off, dst.c_stride, dst.h, dst.w, 0)
        op.cout = cout_p
        if res is not None:
            op.has_res = 1
            op.res = View(res.buf, res.c_off, res.c_stride, res.h, res.w, 0)
        lh, lw = src_segs[0].lh, src_segs[0].lw
        op.out_h = (lh + 2 * (k // 2) - k) // s + 1
        op.out_w = (lw + 2 * (k // 2) - k) // s + 1
        assert (op.out_h, op.out_w) == (dst.h, dst.w), (prefix, op.out_h, op.out_w, dst)
        op.k_steps, op.n_tiles = k_steps, n_tiles
        op.w_off = self.add_blob(packed)
        op.b_off = self.add_blob(bias)
        op.t_off = self.add_blob(tab)
        self.ops.append(op)
        self.op_meta.append(op.out_h * op.out_w * w.shape[0] * w.shape[1] * k * k)
        return op

    # -- graph lowering ------------------------------------------------------------
    def _build(self):
        ar = self.ar
        outs: dict[int, list[Seg]] = {}
        h, w = self.in_h, self.in_w
        prev = None
        for Ly in ar.layers:
            def inp(f):
                if f == -1:
                    return prev
                return outs[f]
            if Ly.kind == "Conv" and Ly.i == 0:
                k, s = Ly.args["k"], Ly.args["s"]
                oh, ow = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
                cp = self.phys(Ly.c2)
                buf = self.new_buf(oh, ow, cp)
                wf, bf, _, _, _ = self.fused["model.0"]
                W0 = np.zeros((cp, 3, k, k), np.float32)
                W0[: Ly.c2] = wf.numpy()
                B0 = np.zeros(cp, np.float32)
                B0[: Ly.c2] = bf.numpy()
                op = Op()
                op.kind = YK_K_CONV_INPUT
                op.ksize, op.stride, op.act = k, s, 1
                op.dst = View(buf, 0, cp, oh, ow, 0)
                op.cout = cp
                op.out_h, op.out_w = oh, ow
                op.w_off = self.add_blob(W0)
                op.b_off = self.add_blob(B0)
                op.t_off = op.b_off
                self.ops.append(op)
                self.op_meta.append(oh * ow * Ly.c2 * 3 * k * k)
                out = [Seg(buf, 0, cp, cp, Ly.c2, oh, ow)]
            elif Ly.kind == "Conv":
                src = inp(Ly.f)
                k, s = Ly.args["k"], Ly.args["s"]
                lh, lw = src[0].lh, src[0].lw
                oh, ow = (lh + 2 * (k // 2) - k) // s + 1, (lw + 2 * (k // 2) - k) // s + 1
                cp = self.phys(Ly.c2)
                buf = self.new_buf(oh, ow, cp)
                dst = Seg(buf, 0, cp, cp, Ly.c2, oh, ow)
                self.conv_op(f"model.{Ly.i}", src, dst, list(range(Ly.c2)), cp)
                out = [dst]
            elif Ly.kind == "C2f":
                out = self._c2f(Ly, inp(Ly.f))
            elif Ly.kind == "SPPF":
                out = self._sppf(Ly, inp(Ly.f))
            elif Ly.kind == "Upsample":
                assert Ly.args["scale"] == 2
                out = [replace(s_, up=s_.up + 1) for s_ in inp(Ly.f)]
            elif Ly.kind == "Concat":
                out = [s_ for f in Ly.f for s_ in inp(f)]
            elif Ly.kind == "Detect":
                out = self._detect(Ly, [inp(f) for f in Ly.f])
            else:
                raise ValueError(Ly.kind)
            outs[Ly.i] = out
            self.layer_out[Ly.i] = out
            prev = out

    def _c2f(self, Ly, src):
        c = int(Ly.c2 * 0.5)
        cp = self.phys(c)
        n = Ly.args["n"]
        hh, ww = src[0].lh, src[0].lw
        Y = self.new_buf(hh, ww, (2 + n) * cp)
        ys = [Seg(Y, j * cp, (2 + n) * cp, cp, c, hh, ww) for j in range(2 + n)]
        p = f"model.{Ly.i}"
        self.conv_op(f"{p}.cv1", src, Seg(Y, 0, (2 + n) * cp, 2 * cp, 2 * c, hh, ww),
                     [o if o < c else cp + o - c for o in range(2 * c)], 2 * cp)
        tmp = self.new_buf(hh, ww, cp)
        ts = Seg(tmp, 0, cp, cp, c, hh, ww)
        for j in range(n):
            self.conv_op(f"{p}.m.{j}.cv1", [ys[1 + j]], ts, list(range(c)), cp)
            self.conv_op(f"{p}.m.{j}.cv2", [ts], ys[2 + j], list(range(c)), cp,
                         res=ys[1 + j] if Ly.args["shortcut"] else None)
        c2p = self.phys(Ly.c2)
        ob = self.new_buf(hh, ww, c2p)
        dst = Seg(ob, 0, c2p, c2p, Ly.c2, hh, ww)
        self.conv_op(f"{p}.cv2", ys, dst, list(range(Ly.c2)), c2p)
        return [dst]

    def _sppf(self, Ly, src):
        c_ = Ly.c1 // 2
        cp = self.phys(c_)
        hh, ww = src[0].lh, src[0].lw
        Z = self.new_buf(hh, ww, 4 * cp)
        zs = [Seg(Z, j * cp, 4 * cp, cp, c_, hh, ww) for j in range(4)]
        p = f"model.{Ly.i}"
        self.conv_op(f"{p}.cv1", src, zs[0], list(range(c_)), cp)
        op = Op()
        op.kind = YK_K_SPPF_POOL
        op.n_src = 1
        op.src[0] = View(Z, 0, 4 * cp, hh, ww, 0)
        op.src_ch[0] = cp
        op.dst = View(Z, cp, 4 * cp, hh, ww, 0)
        op.cout = cp
        op.out_h, op.out_w = hh, ww
        assert Ly.args["k"] == 5
        self.ops.append(op)
        self.op_meta.append(0)
        c2p = self.phys(Ly.c2)
        ob = self.new_buf(hh, ww, c2p)
        dst = Seg(ob, 0, c2p, c2p, Ly.c2, hh, ww)
        self.conv_op(f"{p}.cv2", zs, dst, list(range(Ly.c2)), c2p)
        return [dst]

    def _detect(self, Ly, level_in):
        c2b, c3, nc = Ly.args["c2"], Ly.args["c3"], Ly.args["nc"]
        assert nc == 1 and c2b == 64, "decode kernel: single class, 64 box channels"
        c3p = self.phys(c3)
        p = f"model.{Ly.i}"
        anchor_off = 0
        for li, src in enumerate(level_in):
            hh, ww = src[0].lh, src[0].lw
            width = 64 + c3p
            H1 = self.new_buf(hh, ww, width)
            H2 = self.new_buf(hh, ww, width)
            wa, ba, _, _, _ = self.fused[f"{p}.cv2.{li}.0"]
            wb, bb, _, _, _ = self.fused[f"{p}.cv3.{li}.0"]
            wcat, bcat = torch.cat([wa, wb]), torch.cat([ba, bb])
            omap = list(range(64)) + [64 + o for o in range(c3)]
            self.fused[f"{p}.head.{li}.0"] = (wcat, bcat, 3, 1, True)
            self.conv_op(f"{p}.head.{li}.0", src, Seg(H1, 0, width, width, 64 + c3, hh, ww), omap, width)
            self.conv_op(f"{p}.cv2.{li}.1", [Seg(H1, 0, width, 64, 64, hh, ww)], Seg(H2, 0, width, 64, 64, hh, ww),
                         list(range(64)), 64)
            self.conv_op(f"{p}.cv3.{li}.1", [Seg(H1, 64, width, c3p, c3, hh, ww)],
                         Seg(H2, 64, width, c3p, c3, hh, ww), list(range(c3)), c3p)
            wbox, bbox, _, _, _ = self.fused[f"{p}.cv2.{li}.2"]
            _, packed, bias, _, k_steps, n_tiles = self.pack(wbox, bbox, [Seg(H2, 0, width, 64, 64, hh, ww)],
                                                             list(range(64)), 64)
            wcls, bcls, _, _, _ = self.fused[f"{p}.cv3.{li}.2"]
            wc = np.zeros(c3p + 4, np.float32)
            wc[:c3] = wcls.numpy().reshape(-1)
            wc[c3p] = float(bcls.numpy().reshape(-1)[0])
            op = Op()
            op.kind = YK_K_DETECT
            op.n_src = 1
            op.src[0] = View(H2, 0, width, hh, ww, 0)
            op.src_ch[0] = 64
            op.dst = View(H2, 0, width, hh, ww, 0)
            op.out_h, op.out_w = hh, ww
            op.k_steps, op.n_tiles = k_steps, n_tiles
            op.w_off = self.add_blob(packed)
            op.b_off = self.add_blob(bias)
            op.t_off = op.b_off
            op.det_stride = self.strides[li]
            op.det_anchor_off = anchor_off
            op.det_cls_off = 64
            op.det_cls_ch = c3p
            op.det_wc_off = self.add_blob(wc)
            self.ops.append(op)
            self.op_meta.append(hh * ww * (64 * 64 + c3))
            anchor_off += hh * ww
        self.n_anchors = anchor_off
        return []

    def op_flops(self, B: int) -> list:
        """Algorithmic FLOPs of each op for a batch of B frames (2*MACs of the reference's
        logical, unpadded conv; 0 for pooling; the Detect op counts its 1x1 box/cls convs)."""
        out = []
        for op, meta in zip(self.ops, self.op_meta):
            out.append(2 * B * meta)
        return out + [0]

    # -- device model ----------------------------------------------------------------
    def desc(self):
        self._ops_arr = (Op * len(self.ops))(*self.ops)
        self._bufs_arr = (C.c_int64 * len(self.buf_elems))(*self.buf_elems)
        d = ModelDesc()
        d.act_dtype = ACT[self.dtype]
        d.max_batch = self.max_batch
        d.frame_h, d.frame_w = self.frame_h, self.frame_w
        d.in_h, d.in_w = self.in_h, self.in_w
        d.pad_top, d.pad_left = self.pad_top, self.pad_left
        d.n_anchors, d.nc, d.max_det = self.n_anchors, self.ar.nc, self.max_det
        d.n_bufs = len(self.buf_elems)
        d.buf_elems = C.cast(self._bufs_arr, C.POINTER(C.c_int64))
        d.n_ops = len(self.ops)
        d.ops = C.cast(self._ops_arr, C.POINTER(Op))
        lb = self.lb
        d.rs_mode, d.rs_w, d.rs_h = lb["mode"], lb["new_w"], lb["new_h"]
        d.box_pad_x, d.box_pad_y, d.box_gain = lb["pad_x"], lb["pad_y"], lb["gain"]
        d.rs_tab_off = self.rs_tab_off
        return d


    def export_engine(self, path: str, plan=None, plan_batch: int = 0) -> None:
        """Write this program as an engine file (include/yk.h, yk_model_load): a C host creates
        the model from it without Python.  plan: get_plan()-style [[kind, nnt, npt], ...] per op
        (kind -1 entries are skipped), applied at plan_batch."""
        import struct

        d = self.desc()
        raw = ModelDesc.from_buffer_copy(bytes(d))
        raw.buf_elems = None
        raw.ops = None
        entries = []
        if plan is not None:
            for i, (kind, nnt, npt) in enumerate(plan):
                if kind >= 0 and self.ops[i].kind == YK_K_CONV:
                    entries.append((i, int(kind), int(nnt), int(npt)))
        if entries and not 1 <= plan_batch <= self.max_batch:
            raise ValueError(f"plan_batch must be in [1, {self.max_batch}]")
        head = struct.pack("<8s8iq", b"YKENGINE", 1, C.sizeof(ModelDesc), C.sizeof(Op), len(self.buf_elems),
                           len(self.ops), int(plan_batch), len(entries), 0, len(self.blob))
        with open(path, "wb") as f:
            f.write(head)
            f.write(bytes(raw))
            f.write(np.asarray(self.buf_elems, np.int64).tobytes())
            f.write(bytes((Op * len(self.ops))(*self.ops)))
            f.write(bytes(self.blob))
            if entries:
                f.write(np.asarray(entries, np.int32).tobytes())


class EngineModel:
    """A model created from an engine file by the library itself (yk_model_load): no Program on
    the Python side; frame size and batch come from the file."""

    def __init__(self, path: str | None, device: int = 0, _handle=None):
        self.device = int(device)
        if _handle is not None:
            self._h = _handle
            return
        h = C.c_void_p()
        L.check(L.lib().yk_model_load(L.context(self.device), str(path).encode(), C.byref(h)), "yk_model_load")
        self._h = h

    @classmethod
    def from_state_dict(cls, sd: dict, scale: str, dtype: str, frame_h: int, frame_w: int, imgsz: int = 640,
                        max_batch: int = 8, device: int = 0):
        """The detector built by the library from a raw fp32 state dict (yk_model_load_weights:
        parse_model rules, BN fold and packing in C++, csrc/program.cpp) -- no Program."""
        w, keep = L.weights_struct(sd)
        h = C.c_void_p()
        L.check(L.lib().yk_model_load_weights(L.context(int(device)), C.byref(w), str(scale)[:1].encode(), ACT[dtype],
                                              int(frame_h), int(frame_w), int(imgsz), int(max_batch), C.byref(h)),
                "yk_model_load_weights")
        del keep
        return cls(None, device, _handle=h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.lib().yk_model_destroy(h)
            except Exception:
                pass
            self._h = None

    def detect(self, frames: torch.Tensor, conf=0.25, iou=0.7, max_det=300):
        B = frames.shape[0]
        dets = torch.empty((B, max_det, 6), dtype=torch.float32, device=frames.device)
        counts = torch.empty(B, dtype=torch.int32, device=frames.device)
        L.check(L.lib().yk_detect(self._h, L.ptr(frames), int(B), C.c_float(conf), C.c_float(iou), int(max_det),
                                  L.ptr(dets), L.ptr(counts), L.current_stream(self.device)), "yk_detect")
        return dets, counts


class DeviceModel:
    """A Program instantiated on one GPU (yk_model)."""

    def __init__(self, prog: Program, device: int = 0):
        self.prog, self.device = prog, int(device)
        ctx = L.context(self.device)
        d = prog.desc()
        blob = (C.c_char * len(prog.blob)).from_buffer(prog.blob)
        h = C.c_void_p()
        L.check(L.lib().yk_model_create(ctx, C.byref(d), blob, len(prog.blob), C.byref(h)), "yk_model_create")
        self._h = h
        dets, counts = C.c_void_p(), C.c_void_p()
        L.check(L.lib().yk_model_outputs(h, C.byref(dets), C.byref(counts)), "yk_model_outputs")
        self.dets_ptr, self.counts_ptr = dets.value, counts.value

    def __del__(self):
        h = getattr(self, "_h", None)
        try:
            if h is not None and L._lib is not None:
                L.lib().yk_model_destroy(h)
        except Exception:  # interpreter shutdown
            pass
        self._h = None

    @property
    def handle(self):
        return self._h

    def detect(self, frames: torch.Tensor, conf=0.25, iou=0.7, max_det=300, dets: torch.Tensor | None = None,
               counts: torch.Tensor | None = None, graph: bool = False, stream=None):
        """frames: uint8 device tensor [B, H, W, 3] (BGR).  Returns (dets [B, max_det, 6], counts [B])."""
        p = self.prog
        if frames.dtype != torch.uint8 or frames.dim() != 4 or tuple(frames.shape[1:]) != (p.frame_h, p.frame_w, 3):
            raise ValueError(f"frames must be uint8 [B, {p.frame_h}, {p.frame_w}, 3], got {tuple(frames.shape)}")
        if not frames.is_contiguous():
            raise ValueError("frames must be contiguous")
        B = frames.shape[0]
        dev = frames.device
        if dets is None:
            dets = torch.empty((B, max_det, 6), dtype=torch.float32, device=dev)
        if counts is None:
            counts = torch.empty(B, dtype=torch.int32, device=dev)
        st = L.current_stream(self.device) if stream is None else C.c_void_p(stream)
        fn = L.lib().yk_detect_graph if graph else L.lib().yk_detect
        L.check(fn(self._h, L.ptr(frames), int(B), C.c_float(conf), C.c_float(iou), int(max_det), L.ptr(dets),
                   L.ptr(counts), st), "yk_detect")
        return dets, counts

    def nms(self, rows: torch.Tensor, counts: torch.Tensor, iou=0.7, max_det=300, stream=None):
        """yk_nms: TorchNMS.nms (+ max_nms / max_det / scale / clip) of the model's nms_kernel on
        given boxes.  rows: float32 device [B, R, >=5] (x1 y1 x2 y2 score, network-input pixels),
        counts: int32 device [B].  Returns (dets [B, max_det, 6], counts [B], keep [B, max_det]:
        input row of every output row)."""
        if rows.dtype != torch.float32 or rows.dim() != 3 or rows.shape[2] < 5 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous float32 tensor [B, R, >=5]")
        if counts.dtype != torch.int32 or counts.shape != (rows.shape[0],):
            raise ValueError("counts must be an int32 tensor [B]")
        B, R, S = rows.shape
        dev = rows.device
        dets = torch.zeros((B, max_det, 6), dtype=torch.float32, device=dev)
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        keep = torch.full((B, max_det), -1, dtype=torch.int32, device=dev)
        st = L.current_stream(self.device) if stream is None else C.c_void_p(stream)
        L.check(L.lib().yk_nms(self._h, L.ptr(rows), int(S), int(R), L.ptr(counts), int(B), C.c_float(iou),
                               int(max_det), L.ptr(dets), L.ptr(cnt), L.ptr(keep), st), "yk_nms")
        return dets, cnt, keep

    def nms_candidates(self, B: int, iou=0.7, max_det=300):
        """yk_nms_candidates: the NMS stage alone on the model's current candidate buffers."""
        dev = torch.device("cuda", self.device)
        dets = torch.zeros((B, max_det, 6), dtype=torch.float32, device=dev)
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        keep = torch.full((B, max_det), -1, dtype=torch.int32, device=dev)
        L.check(L.lib().yk_nms_candidates(self._h, int(B), C.c_float(iou), int(max_det), L.ptr(dets), L.ptr(cnt),
                                          L.ptr(keep), L.current_stream(self.device)), "yk_nms_candidates")
        return dets, cnt, keep

    def nms_stats(self, reset: bool = False):
        """(images that took TorchNMS's :291-296 early exit with boxes left, images processed)."""
        out = np.zeros(2, np.int64)
        L.check(L.lib().yk_model_nms_stats(self._h, L.ptr(out), int(bool(reset)), L.current_stream(self.device)),
                "yk_model_nms_stats")
        return int(out[0]), int(out[1])

    def check(self):
        """Synchronise and raise YKError if a device-side error was flagged (yk_model_check)."""
        L.check(L.lib().yk_model_check(self._h, L.current_stream(self.device)), "yk_model_check")

    def set_lanes(self, lanes: int):
        """Streams the op DAG is scheduled onto (1 = strictly sequential, the reference's order)."""
        L.check(L.lib().yk_model_set_lanes(self._h, int(lanes)), "yk_model_set_lanes")

    def autotune(self, frames: torch.Tensor, conf=0.25, reps: int = 10):
        """Pick the fastest conv kernel variant per op for this batch size (yk_model_autotune)."""
        L.check(L.lib().yk_model_autotune(self._h, L.ptr(frames), int(frames.shape[0]), C.c_float(conf), int(reps),
                                          L.current_stream(self.device)), "yk_model_autotune")
        torch.cuda.synchronize(self.device)

    def set_plan(self, batch: int, kind: int, nnt: int = 0, npt: int = 0, op: int = -1):
        """Force the conv kernel (-1 heuristic, 0 direct, 1 LDS-tiled, 2 split-K nnt x npt)."""
        L.check(L.lib().yk_model_set_plan(self._h, int(op), int(batch), int(kind), int(nnt), int(npt)),
                "yk_model_set_plan")

    def get_plan(self):
        """(batch, [[kind, nnt, npt] per op]) of the current conv plan (autotune result)."""
        n = len(self.prog.ops)
        plan, b = np.zeros(3 * n, np.int32), np.zeros(1, np.int32)
        L.check(L.lib().yk_model_get_plan(self._h, L.ptr(plan), L.ptr(b)), "yk_model_get_plan")
        return int(b[0]), plan.reshape(n, 3).tolist()

    def load_plan(self, batch: int, plan):
        """Re-apply a plan from get_plan() (per conv op; kind -1 keeps the heuristic)."""
        for i, (kind, nnt, npt) in enumerate(plan):
            if self.prog.ops[i].kind == YK_K_CONV:
                self.set_plan(batch, kind, nnt, npt, op=i)

    def set_schedule(self, groups: int, lanes: int):
        """Cut the batch into `groups` independent sub-batches, each on `lanes` streams."""
        L.check(L.lib().yk_model_set_schedule(self._h, int(groups), int(lanes)), "yk_model_set_schedule")
        self.groups = int(groups)

    def schedule(self):
        """(lane per task, cross-lane waits per task) of the current DAG schedule (op-major)."""
        n = len(self.prog.ops) * getattr(self, "groups", 1)
        lane, waits = np.zeros(n, np.int32), np.zeros(n, np.int32)
        L.check(L.lib().yk_model_get_schedule(self._h, L.ptr(lane), L.ptr(waits)), "yk_model_get_schedule")
        return lane, waits

    def profile(self, frames: torch.Tensor, conf=0.25, iou=0.7, max_det=300, reps: int = 5):
        """Per-op device milliseconds (hipEvents, `reps` back-to-back launches each) and the
        kernel instantiation each op launches.  Returns list of (op_index, kind, kernel, ms)."""
        n = len(self.prog.ops)
        ms = np.zeros(n + 1, np.float32)
        B = frames.shape[0]
        L.check(L.lib().yk_model_profile(self._h, L.ptr(frames), int(B), C.c_float(conf), C.c_float(iou), int(max_det),
                                         int(reps), L.ptr(ms), L.current_stream(self.device)), "yk_model_profile")
        out = []
        buf = C.create_string_buffer(128)
        for i in range(n + 1):
            L.check(L.lib().yk_model_op_kernel(self._h, i, buf, 128), "yk_model_op_kernel")
            kind = self.prog.ops[i].kind if i < n else -1
            out.append((i, kind, buf.value.decode(), float(ms[i])))
        return out

    def candidates(self, B: int):
        """Pre-NMS candidates of the last detect() as a [B, n_anchors, 6] view + counts (copies)."""
        cand, cnt = C.c_void_p(), C.c_void_p()
        L.check(L.lib().yk_model_candidates(self._h, C.byref(cand), C.byref(cnt)), "yk_model_candidates")
        A_ = self.prog.n_anchors
        torch.cuda.synchronize(self.device)
        host = np.zeros((self.prog.max_batch, A_, 6), np.float32)
        hc = np.zeros(self.prog.max_batch, np.int32)
        _memcpy_d2h(host, cand.value)
        _memcpy_d2h(hc, cnt.value)
        return host[:B], hc[:B]

    def buffer(self, idx: int, B: int):
        """Activation buffer `idx` as a host float32 array [B, elems] (debug / parity)."""
        ptr = C.c_void_p()
        L.check(L.lib().yk_model_buffer(self._h, int(idx), C.byref(ptr)), "yk_model_buffer")
        torch.cuda.synchronize(self.device)
        n = self.prog.buf_elems[idx] * B
        if self.prog.dtype == "bf16":
            raw = np.zeros(n, np.int16)
            _memcpy_d2h(raw, ptr.value)
            out = torch.from_numpy(raw).view(torch.bfloat16).float().numpy()
        elif self.prog.dtype == "fp16":
            raw = np.zeros(n, np.float16)
            _memcpy_d2h(raw, ptr.value)
            out = raw.astype(np.float32)
        elif self.prog.dtype == "fp8":
            raw = np.zeros(n, np.uint8)
            _memcpy_d2h(raw, ptr.value)
            out = torch.from_numpy(raw).view(torch.float8_e4m3fn).float().numpy()
        else:
            out = np.zeros(n, np.float32)
            _memcpy_d2h(out, ptr.value)
        return out.reshape(B, -1)

    def letterboxed(self, B: int) -> np.ndarray:
        """The letterboxed uint8 input [B, in_h, in_w, 3] of the last detect() (resizing models)."""
        ptr = C.c_void_p()
        L.check(L.lib().yk_model_buffer(self._h, -1, C.byref(ptr)), "yk_model_buffer")
        if not ptr.value:
            raise L.YKError("this model's frames need no LetterBox resize")
        torch.cuda.synchronize(self.device)
        out = np.zeros((B, self.prog.in_h, self.prog.in_w, 3), np.uint8)
        _memcpy_d2h(out, ptr.value)
        return out

    def layer_nchw(self, i: int, B: int) -> torch.Tensor:
        """Logical output of graph layer i as an NCHW float tensor (debug / parity)."""
        segs = self.prog.layer_out[i]
        parts = []
        for s in segs:
            a = self.buffer(s.buf, B).reshape(B, s.h, s.w, s.c_stride)[..., s.c_off:s.c_off + s.cl]
            t = torch.from_numpy(np.ascontiguousarray(a)).permute(0, 3, 1, 2)
            if s.up:
                t = torch.nn.functional.interpolate(t, scale_factor=2 ** s.up, mode="nearest")
            parts.append(t)
        return torch.cat(parts, 1)


def _memcpy_d2h(dst: np.ndarray, src_ptr: int):
    L.check(L.lib().yk_memcpy_d2h(L.ptr(dst), C.c_void_p(src_ptr), C.c_int64(dst.nbytes)), "yk_memcpy_d2h")
