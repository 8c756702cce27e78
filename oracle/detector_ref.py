"""torch-CPU restatement of the YOLOv8-small+P2 predict path (TEST ORACLE ONLY).

Follows the reference's modules operation by operation, fp32 ATen on the CPU:
  preprocess      engine/predictor.py:152-204 + data/augment.py:1667-1744 (LetterBox; only the
                  no-resize case r == 1, since cv2 is not available here)
  graph           nn/tasks.py:159-188 (_predict_once) over the parse_model layer list
  Conv (fused)    nn/modules/conv.py:39-93 forward_fuse, utils/torch_utils.py:255-286
  C2f/Bottleneck  nn/modules/block.py:294-322, 470-492
  SPPF            nn/modules/block.py:216-238
  Detect          nn/modules/head.py:116-187 (legacy v8 head), DFL block.py:58-82,
                  make_anchors / dist2bbox utils/tal.py:367-391
  NMS             utils/nms.py:13-167 (non_max_suppression) + 237-304 (TorchNMS.nms,
                  with its "no overlap -> keep all remaining" early exit)
  results         models/yolo/detect/predict.py:111-125, utils/ops.py:105-184 (scale/clip)

The layer list itself comes from the caller (``layers``: the parsed topology as plain
tuples) so the graph builder under test is checked independently: this module only
executes a layer list against a state dict.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

REG_MAX = 16


def fuse(sd, prefix, eps=1e-3):
    """fuse_conv_and_bn (torch_utils.py:255-286), verbatim arithmetic."""
    w = sd[f"{prefix}.conv.weight"].float()
    g, b = sd[f"{prefix}.bn.weight"].float(), sd[f"{prefix}.bn.bias"].float()
    m, v = sd[f"{prefix}.bn.running_mean"].float(), sd[f"{prefix}.bn.running_var"].float()
    w_bn = torch.diag(g.div(torch.sqrt(eps + v)))
    wf = torch.mm(w_bn, w.view(w.shape[0], -1)).view(w.shape)
    b_conv = torch.zeros(w.shape[0])
    b_bn = b - g.mul(m).div(torch.sqrt(v + eps))
    bf = torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn
    return wf, bf


class RefDetector:
    """Executes a parsed layer list.  ``layers``: list of (i, f, kind, args) where args holds
    k/s (Conv), n/shortcut/c (C2f), k (SPPF), scale (Upsample), nc (Detect)."""

    def __init__(self, layers, sd, strides):
        self.layers, self.sd, self.strides = layers, sd, strides
        self.save = sorted({x % i for (i, f, _, _) in layers for x in ([f] if isinstance(f, int) else f) if x != -1})
        self._w = {}

    def conv(self, x, p, k, s, act=True):
        if p not in self._w:
            self._w[p] = fuse(self.sd, p)
        w, b = self._w[p]
        y = F.conv2d(x, w, b, s, k // 2)
        return F.silu(y) if act else y

    def c2f(self, x, p, n, shortcut, c):
        y = list(self.conv(x, f"{p}.cv1", 1, 1).chunk(2, 1))
        for j in range(n):
            t = self.conv(self.conv(y[-1], f"{p}.m.{j}.cv1", 3, 1), f"{p}.m.{j}.cv2", 3, 1)
            y.append(y[-1] + t if shortcut else t)
        return self.conv(torch.cat(y, 1), f"{p}.cv2", 1, 1)

    def sppf(self, x, p, k):
        y = [self.conv(x, f"{p}.cv1", 1, 1)]
        for _ in range(3):
            y.append(F.max_pool2d(y[-1], k, 1, k // 2))
        return self.conv(torch.cat(y, 1), f"{p}.cv2", 1, 1)

    def detect(self, xs, p, nc):
        outs = []
        for li, x in enumerate(xs):
            a = self.conv(self.conv(x, f"{p}.cv2.{li}.0", 3, 1), f"{p}.cv2.{li}.1", 3, 1)
            a = F.conv2d(a, self.sd[f"{p}.cv2.{li}.2.weight"].float(), self.sd[f"{p}.cv2.{li}.2.bias"].float())
            c = self.conv(self.conv(x, f"{p}.cv3.{li}.0", 3, 1), f"{p}.cv3.{li}.1", 3, 1)
            c = F.conv2d(c, self.sd[f"{p}.cv3.{li}.2.weight"].float(), self.sd[f"{p}.cv3.{li}.2.bias"].float())
            outs.append(torch.cat((a, c), 1))
        return self.inference(outs, nc, p), outs

    def inference(self, xs, nc, p):
        no = nc + 4 * REG_MAX
        b = xs[0].shape[0]
        x_cat = torch.cat([xi.view(b, no, -1) for xi in xs], 2)
        # make_anchors (tal.py:367-380)
        pts, sts = [], []
        for xi, st in zip(xs, self.strides):
            h, w = xi.shape[2:]
            sx = torch.arange(w, dtype=torch.float32) + 0.5
            sy = torch.arange(h, dtype=torch.float32) + 0.5
            sy, sx = torch.meshgrid(sy, sx, indexing="ij")
            pts.append(torch.stack((sx, sy), -1).view(-1, 2))
            sts.append(torch.full((h * w, 1), st, dtype=torch.float32))
        anchors, strides = torch.cat(pts).transpose(0, 1), torch.cat(sts).transpose(0, 1)
        box, cls = x_cat.split((4 * REG_MAX, nc), 1)
        # DFL (block.py:77-80)
        a = box.shape[2]
        dfl_w = self.sd[f"{p}.dfl.conv.weight"].float()
        d = F.conv2d(box.view(b, 4, REG_MAX, a).transpose(2, 1).softmax(1), dfl_w).view(b, 4, a)
        # dist2bbox (tal.py:383-391), xywh
        lt, rb = d.chunk(2, 1)
        x1y1 = anchors.unsqueeze(0) - lt
        x2y2 = anchors.unsqueeze(0) + rb
        dbox = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1) * strides
        return torch.cat((dbox, cls.sigmoid()), 1)

    @torch.no_grad()
    def forward(self, x, keep_all=False):
        y = []
        out = None
        self.outputs = {}
        for (i, f, kind, args) in self.layers:
            if f != -1:
                inp = y[f] if isinstance(f, int) else [x if j == -1 else y[j] for j in f]
            else:
                inp = x
            p = f"model.{i}"
            if kind == "Conv":
                x = self.conv(inp, p, args["k"], args["s"])
            elif kind == "C2f":
                x = self.c2f(inp, p, args["n"], args["shortcut"], args["c"])
            elif kind == "SPPF":
                x = self.sppf(inp, p, args["k"])
            elif kind == "Upsample":
                x = F.interpolate(inp, scale_factor=args["scale"], mode="nearest")
            elif kind == "Concat":
                x = torch.cat(inp, 1)
            elif kind == "Detect":
                out = self.detect(inp, p, args["nc"])
                x = out
            y.append(x if i in self.save else None)
            if keep_all:
                self.outputs[i] = x
        return out


def preprocess(frames, imgsz=640, stride=32):
    """BGR HWC uint8 frames (same shape) -> (B,3,H,W) float32 RGB/255 after LetterBox(auto)
    (engine/predictor.py:152-204); a frame off the network scale is resized with the
    oracle's cv2 INTER_LINEAR restatement (oracle/letterbox_ref.py, parity with cv2 unpinned)."""
    import numpy as np

    from .letterbox_ref import letterbox

    ims = [letterbox(f, imgsz, stride) for f in frames]
    im = np.stack(ims)[..., ::-1].transpose(0, 3, 1, 2)
    t = torch.from_numpy(np.ascontiguousarray(im)).float()
    t /= 255
    return t


def torch_nms(boxes, scores, iou_threshold):
    """TorchNMS.nms (nms.py:237-304), including the early exit of :291-296."""
    if boxes.numel() == 0:
        return torch.empty((0,), dtype=torch.int64)
    x1, y1, x2, y2 = boxes.unbind(1)
    areas = (x2 - x1) * (y2 - y1)
    _, order = scores.sort(stable=True, dim=0, descending=True)
    keep = torch.zeros(order.numel(), dtype=torch.int64)
    k = 0
    while order.numel() > 0:
        i = order[0]
        keep[k] = i
        k += 1
        if order.numel() == 1:
            break
        rest = order[1:]
        xx1 = torch.maximum(x1[i], x1[rest])
        yy1 = torch.maximum(y1[i], y1[rest])
        xx2 = torch.minimum(x2[i], x2[rest])
        yy2 = torch.minimum(y2[i], y2[rest])
        inter = (xx2 - xx1).clamp_(min=0) * (yy2 - yy1).clamp_(min=0)
        if inter.sum() == 0:
            keep[k:k + rest.numel()] = rest
            k += rest.numel()
            break
        iou = inter / (areas[i] + areas[rest] - inter)
        order = rest[iou <= iou_threshold]
    return keep[:k]


def non_max_suppression(pred, conf_thres=0.25, iou_thres=0.7, max_det=300, max_nms=30000, max_wh=7680,
                        agnostic=False):
    """non_max_suppression (nms.py:13-167), single-label path.  Sorting is made stable
    (score desc, then anchor order) -- torch's default CPU sort is unstable on exact ties,
    so the reference's order among equal scores is implementation-defined."""
    assert 0 <= conf_thres <= 1 and 0 <= iou_thres <= 1
    bs, nc = pred.shape[0], pred.shape[1] - 4
    xc = pred[:, 4:4 + nc].amax(1) > conf_thres
    pred = pred.transpose(-1, -2).clone()
    xy, wh = pred[..., :2], pred[..., 2:4] / 2
    pred[..., :4] = torch.cat((xy - wh, xy + wh), -1)
    out = [torch.zeros((0, 6))] * bs
    for xi, x in enumerate(pred):
        x = x[xc[xi]]
        if not x.shape[0]:
            continue
        box, cls = x[:, :4], x[:, 4:4 + nc]
        conf, j = cls.max(1, keepdim=True)
        x = torch.cat((box, conf, j.float()), 1)[conf.view(-1) > conf_thres]
        if not x.shape[0]:
            continue
        if x.shape[0] > max_nms:
            x = x[x[:, 4].sort(descending=True, stable=True)[1][:max_nms]]
        c = x[:, 5:6] * (0 if agnostic else max_wh)
        i = torch_nms(x[:, :4] + c, x[:, 4], iou_thres)[:max_det]
        out[xi] = x[i]
    return out


def scale_clip(pred, img_hw, orig_hw):
    """scale_boxes + clip_boxes (ops.py:105-184) for LetterBox-centred inputs."""
    gain = min(img_hw[0] / orig_hw[0], img_hw[1] / orig_hw[1])
    px = round((img_hw[1] - orig_hw[1] * gain) / 2 - 0.1)
    py = round((img_hw[0] - orig_hw[0] * gain) / 2 - 0.1)
    b = pred[:, :4]
    b[:, 0] -= px
    b[:, 1] -= py
    b[:, 2] -= px
    b[:, 3] -= py
    b /= gain
    b[:, 0].clamp_(0, orig_hw[1])
    b[:, 1].clamp_(0, orig_hw[0])
    b[:, 2].clamp_(0, orig_hw[1])
    b[:, 3].clamp_(0, orig_hw[0])
    return pred


def predict(det: RefDetector, frames, conf=0.25, iou=0.7, max_det=300, imgsz=640):
    """Model.predict for a list of same-shape BGR frames -> list of (N, 6) float32 tensors
    [x1, y1, x2, y2, conf, cls] in original-image pixels (Results.boxes.data)."""
    im = preprocess(frames, imgsz)
    y, _ = det.forward(im)
    out = non_max_suppression(y, conf, iou, max_det)
    return [scale_clip(p, im.shape[2:], frames[0].shape[:2]) for p in out], y


# ---------------------------------------------------------------- FP8 build restatement
def e4m3(t):
    """Round to OCP e4m3 (float8_e4m3fn), saturating at +-448, as the FP8 build stores
    every activation; returns float32 values."""
    return t.float().clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()


def fp8_weights(w):
    """Per-output-channel e4m3 weights of the FP8 build: scale = 448 / max|w[o]| (f32),
    Wq = e4m3(w * scale), dequant dq = 1 / scale (f32).  Returns (Wq, dq)."""
    amax = w.abs().flatten(1).amax(1)
    # true f32 divisions (a python scalar over a tensor is reciprocal() * scalar in torch)
    scale = torch.where(amax > 0, torch.full_like(amax, 448.0) / amax.clamp_min(1e-30), torch.ones_like(amax)).float()
    dq = (torch.ones_like(scale) / scale).float()
    return e4m3(w * scale.view(-1, 1, 1, 1)), dq


class RefDetectorFP8(RefDetector):
    """The reference graph (same modules as RefDetector) in the FP8 build's arithmetic, the
    checker for the MI355X fp8 path (BASELINE config 5).  Not a reference-parity claim: the
    reference is fp32; this restates the quantisation the fp8 build applies on top of it:

      * conv weights: per-output-channel e4m3 (fp8_weights), y = conv(x, Wq) * dq + b;
      * every stored activation (conv output after SiLU and the Bottleneck add) is e4m3;
      * layer 0 keeps the bf16 first conv of the production build (raw uint8 values x
        bf16(w * (1/255)), f32 accumulate), its output stored e4m3;
      * Detect: box 1x1 with e4m3 weights (not stored: f32 logits), class 1x1 in f32;
        DFL / dist2bbox / sigmoid as RefDetector.
    Products of e4m3 values are exact in f32, so the GPU and this restatement differ only in
    f32 summation order and the SiLU's exp/rcp, which moves a few values across an e4m3
    rounding boundary per layer."""

    def __init__(self, layers, sd, strides):
        super().__init__(layers, sd, strides)
        self._q = {}

    def _qw(self, p):
        if p not in self._q:
            if p not in self._w:
                self._w[p] = fuse(self.sd, p)
            w, b = self._w[p]
            wq, dq = fp8_weights(w)
            self._q[p] = (wq, dq, b)
        return self._q[p]

    def conv(self, x, p, k, s, act=True, res=None):
        if p == "model.0":
            w, b = self._w.setdefault(p, fuse(self.sd, p))
            raw = torch.round(x * 255.0)
            w0 = (w * torch.tensor(1.0 / 255.0, dtype=torch.float32)).to(torch.bfloat16).float()
            y = F.conv2d(raw, w0, b, s, k // 2)
        else:
            wq, dq, b = self._qw(p)
            y = F.conv2d(x, wq, None, s, k // 2) * dq.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)
        if act:
            y = F.silu(y)
        if res is not None:
            y = res + y
        return e4m3(y)

    def c2f(self, x, p, n, shortcut, c):
        y = list(self.conv(x, f"{p}.cv1", 1, 1).chunk(2, 1))
        for j in range(n):
            t = self.conv(y[-1], f"{p}.m.{j}.cv1", 3, 1)
            y.append(self.conv(t, f"{p}.m.{j}.cv2", 3, 1, res=y[-1] if shortcut else None))
        return self.conv(torch.cat(y, 1), f"{p}.cv2", 1, 1)

    def detect(self, xs, p, nc):
        outs = []
        for li, x in enumerate(xs):
            a = self.conv(self.conv(x, f"{p}.cv2.{li}.0", 3, 1), f"{p}.cv2.{li}.1", 3, 1)
            wb, bb = self.sd[f"{p}.cv2.{li}.2.weight"].float(), self.sd[f"{p}.cv2.{li}.2.bias"].float()
            wq, dq = fp8_weights(wb)
            a = F.conv2d(a, wq) * dq.view(1, -1, 1, 1) + bb.view(1, -1, 1, 1)
            c = self.conv(self.conv(x, f"{p}.cv3.{li}.0", 3, 1), f"{p}.cv3.{li}.1", 3, 1)
            c = F.conv2d(c, self.sd[f"{p}.cv3.{li}.2.weight"].float(), self.sd[f"{p}.cv3.{li}.2.bias"].float())
            outs.append(torch.cat((a, c), 1))
        return self.inference(outs, nc, p), outs
