"""Model weights: synthetic (seeded) state dicts in the reference's naming, and the
Conv+BN fusion of ``fuse_conv_and_bn`` (ultralytics/utils/torch_utils.py:255-286).

The reference's trained ``best.pt`` is absent, so benchmarks and
parity runs use seeded random weights with the reference's module shapes.  With
``planted=True`` a hand-set pass-through channel carries local image brightness from the
input to the P2 Detect classification logit, so the detector really fires on the bright
synthetic targets (SURVEY §8d option (i)); DFL logits are peaked so boxes have a fixed
nominal size, and the P3-P5 classifiers never fire.  Every other weight stays random,
so every conv does its full work.
"""
from __future__ import annotations

import math

import torch

from . import arch as A

BN_EPS = 1e-3  # initialize_weights (ultralytics/utils/torch_utils.py:488-498)


def synthetic_state_dict(ar: A.Arch, seed: int = 0, planted: bool = True, box_bins: float = 12.0,
                         p2_gain: float = 1.0, p2_threshold: float = 5.0, dog: float = 1.0) -> dict:
    g = torch.Generator().manual_seed(seed)

    def rn(*shape, std=1.0):
        return torch.randn(*shape, generator=g) * std

    def ru(lo, hi, *shape):
        return lo + (hi - lo) * torch.rand(*shape, generator=g)

    sd = {}
    strides = A.detect_strides(ar)
    for p, c1, c2, k, s, bn in A.conv_specs(ar):
        fan = c1 * k * k
        if bn:
            sd[f"{p}.conv.weight"] = rn(c2, c1, k, k, std=1.0 / math.sqrt(fan))
            sd[f"{p}.bn.weight"] = ru(0.8, 1.2, c2)
            sd[f"{p}.bn.bias"] = rn(c2, std=0.05)
            sd[f"{p}.bn.running_mean"] = rn(c2, std=0.05)
            sd[f"{p}.bn.running_var"] = ru(0.8, 1.2, c2)
            sd[f"{p}.bn.num_batches_tracked"] = torch.tensor(0)
        else:
            sd[f"{p}.weight"] = rn(c2, c1, k, k, std=0.02)
            lvl = int(p.split(".")[-2])
            if ".cv2." in p:  # box branch: bias 1.0 (Detect.bias_init, head.py:189-200)
                sd[f"{p}.bias"] = torch.ones(c2)
            else:
                sd[f"{p}.bias"] = torch.full((c2,), math.log(5 / ar.nc / (640 / strides[lvl]) ** 2))
    det = ar.layers[-1]
    sd[f"model.{det.i}.dfl.conv.weight"] = torch.arange(A.REG_MAX, dtype=torch.float32).view(1, A.REG_MAX, 1, 1)
    if planted and _is_p2_topology(ar):
        _plant(sd, ar, box_bins, p2_gain, p2_threshold, dog)
    return sd


def _is_p2_topology(ar: A.Arch) -> bool:
    L = ar.layers
    return (len(L) == 26 and L[-1].kind == "Detect" and L[-1].f == [18, 15, 21, 24]
            and L[17].kind == "Concat" and L[17].f == [-1, 2])


def _identity_bn(sd, p, bias=0.0):
    c2 = sd[f"{p}.bn.weight"].shape[0]
    del c2
    sd[f"{p}.bn.weight"][0] = 1.0
    sd[f"{p}.bn.bias"][0] = bias
    sd[f"{p}.bn.running_mean"][0] = 0.0
    sd[f"{p}.bn.running_var"][0] = 1.0 - BN_EPS


def _row0(sd, p, taps):
    """Output channel 0 of conv `p` reads only the given (in_channel, ky, kx, weight) taps."""
    w = sd[f"{p}.conv.weight"]
    w[0].zero_()
    for c, ky, kx, v in taps:
        w[0, c, ky, kx] = v


def _plant(sd, ar, box_bins, gain, thr, dog):
    det = ar.layers[-1]
    c15 = ar.layers[15].c2
    # L0: 3x3x3 mean of the [0,1] image, contrast-stretched (blob ~0.9, background ~0.35)
    _row0(sd, "model.0", [(c, ky, kx, 12.0 / 27.0) for c in range(3) for ky in range(3) for kx in range(3)])
    _identity_bn(sd, "model.0", bias=-4.0)
    _row0(sd, "model.1", [(0, ky, kx, 1.0 / 9.0) for ky in range(3) for kx in range(3)])
    _identity_bn(sd, "model.1")
    for p, src in (("model.2.cv1", 0), ("model.2.cv2", 0), ("model.18.cv1", c15), ("model.18.cv2", 0)):
        _row0(sd, p, [(src, 0, 0, 1.0)])
        _identity_bn(sd, p)
    d = det.i
    # P2 classifier: channel 0 = fine brightness, channel 1 = its 5x5-cell surround;
    # logit = gain * (f0 + dog * (f0 - f1) - thr) peaks at the blob centre (difference of boxes)
    for j in (0, 1):
        p = f"model.{d}.cv3.0.{j}"
        _row0(sd, p, [(0, 1, 1, 1.0)])
        _identity_bn(sd, p)
        w = sd[f"{p}.conv.weight"]
        w[1].zero_()
        w[1, j, :, :] = 1.0 / 9.0
        sd[f"{p}.bn.weight"][1] = 1.0
        sd[f"{p}.bn.bias"][1] = 0.0
        sd[f"{p}.bn.running_mean"][1] = 0.0
        sd[f"{p}.bn.running_var"][1] = 1.0 - BN_EPS
    w = sd[f"model.{d}.cv3.0.2.weight"]
    w.zero_()
    w[0, 0, 0, 0] = gain * (1.0 + dog)
    w[0, 1, 0, 0] = -gain * dog
    sd[f"model.{d}.cv3.0.2.bias"][:] = -gain * thr
    for lvl in range(1, len(det.f)):
        sd[f"model.{d}.cv3.{lvl}.2.weight"].zero_()
        sd[f"model.{d}.cv3.{lvl}.2.bias"][:] = -30.0
    # DFL logits peaked at `box_bins` for every side -> boxes of ~2*box_bins*stride pixels
    bins = torch.arange(A.REG_MAX, dtype=torch.float32)
    logit = -0.5 * (bins - box_bins) ** 2
    for lvl in range(len(det.f)):
        sd[f"model.{d}.cv2.{lvl}.2.bias"][:] = logit.repeat(4)


def _sqrt_f32(x: torch.Tensor) -> torch.Tensor:
    """IEEE (correctly rounded) float32 square root.  torch.sqrt on the CPU goes through MKL's
    vector math here, which misrounds ~0.6% of float32 inputs by one ulp; the C-ABI builder
    (csrc/program.cpp) uses sqrtf, so both hosts fold identical weights."""
    import numpy as np

    return torch.from_numpy(np.sqrt(x.detach().cpu().numpy().astype(np.float32)))


def fuse_conv_bn(w: torch.Tensor, gamma, beta, mean, var, eps: float = BN_EPS):
    """fuse_conv_and_bn (torch_utils.py:255-286) in float32: W' = diag(g/sqrt(eps+var)) W,
    b' = beta - g*mean/sqrt(var+eps) (the conv has no bias).  Every step is one correctly rounded
    float32 operation (the sqrt included, see _sqrt_f32)."""
    sq = _sqrt_f32(var + eps)
    scale = gamma.div(sq)
    wf = (w.reshape(w.shape[0], -1) * scale[:, None]).reshape(w.shape)
    bf = beta - gamma.mul(mean).div(sq)
    return wf, bf


def fused_convs(sd: dict, ar: A.Arch) -> dict:
    """prefix -> (W float32 [c2, c1, k, k], b float32 [c2], k, s, act) after Conv+BN fusion."""
    out = {}
    for p, c1, c2, k, s, bn in A.conv_specs(ar):
        if bn:
            w, b = fuse_conv_bn(sd[f"{p}.conv.weight"].float(), sd[f"{p}.bn.weight"].float(), sd[f"{p}.bn.bias"].float(),
                                sd[f"{p}.bn.running_mean"].float(), sd[f"{p}.bn.running_var"].float())
        else:
            w, b = sd[f"{p}.weight"].float(), sd[f"{p}.bias"].float()
        out[p] = (w.contiguous(), b.contiguous(), k, s, bn)
    return out


def save_raw(path: str, sd: dict) -> None:
    """The state dict as a raw fp32 file for the C-ABI builder (yk_model_load_weights via
    examples/c_host.c): b"YKWTS\\0\\0\\0", int32 version 1, int32 n, then per floating tensor int32
    name length, name, int32 ndim, int64 shape[ndim], float32 data (C order), little-endian."""
    import struct

    import numpy as np

    items = []
    for k, v in sd.items():
        a = v.detach().cpu().float().numpy() if hasattr(v, "detach") else np.asarray(v)
        if a.dtype.kind == "f" and a.ndim <= 4:
            items.append((k, np.ascontiguousarray(a, dtype="<f4")))
    with open(path, "wb") as f:
        f.write(b"YKWTS\0\0\0" + struct.pack("<ii", 1, len(items)))
        for k, a in items:
            name = k.encode()
            f.write(struct.pack("<i", len(name)) + name + struct.pack("<i", a.ndim))
            f.write(struct.pack(f"<{a.ndim}q", *a.shape))
            f.write(a.tobytes())
