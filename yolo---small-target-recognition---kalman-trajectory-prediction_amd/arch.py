"""Model-definition rules of the reference for the detection path.

Restates ``parse_model`` (ultralytics/nn/tasks.py:1524-1700), ``yaml_model_load`` /
``guess_model_scale`` (tasks.py:1703-1740) and the module constructors the P2 model uses
(Conv nn/modules/conv.py:39-93, C2f block.py:294-322, Bottleneck block.py:470-492,
SPPF block.py:216-238, Detect head.py:26-209 with legacy=True for v8 models).

The topology table below encodes ultralytics/cfg/models/v8/yolov8-small.yaml (the
reference's custom 4-scale model with the extra P2 output).  A user YAML with the same
module vocabulary (Conv, C2f, SPPF, nn.Upsample, Concat, Detect) is parsed the same way,
so the standard 3-scale yolov8.yaml works too.
"""
from __future__ import annotations

import math
import os
import re
from dataclasses import dataclass, field

# yolov8-small.yaml (P2..P5 heads), as (from, repeats, module, args)
YOLOV8_SMALL = {
    "nc": 1,
    "scales": {"n": [0.50, 0.375, 1024], "s": [0.67, 0.625, 1024], "m": [1.00, 0.875, 768],
               "l": [1.33, 1.125, 512], "x": [1.67, 1.375, 512]},
    "backbone": [
        [-1, 1, "Conv", [32, 3, 2]],
        [-1, 1, "Conv", [64, 3, 2]],
        [-1, 3, "C2f", [64, True]],
        [-1, 1, "Conv", [128, 3, 2]],
        [-1, 6, "C2f", [128, True]],
        [-1, 1, "Conv", [256, 3, 2]],
        [-1, 6, "C2f", [256, True]],
        [-1, 1, "Conv", [512, 3, 2]],
        [-1, 3, "C2f", [512, True]],
        [-1, 1, "SPPF", [512, 5]],
    ],
    "head": [
        [-1, 1, "nn.Upsample", [None, 2, "nearest"]],
        [[-1, 6], 1, "Concat", [1]],
        [-1, 3, "C2f", [256]],
        [-1, 1, "nn.Upsample", [None, 2, "nearest"]],
        [[-1, 4], 1, "Concat", [1]],
        [-1, 3, "C2f", [128]],
        [-1, 1, "nn.Upsample", [None, 2, "nearest"]],
        [[-1, 2], 1, "Concat", [1]],
        [-1, 3, "C2f", [64]],
        [15, 1, "Conv", [128, 3, 2]],
        [[-1, 12], 1, "Concat", [1]],
        [-1, 3, "C2f", [256]],
        [-1, 1, "Conv", [256, 3, 2]],
        [[-1, 9], 1, "Concat", [1]],
        [-1, 3, "C2f", [512]],
        [[18, 15, 21, 24], 1, "Detect", ["nc"]],
    ],
}
BUILTIN = {"yolov8-small": YOLOV8_SMALL}
REG_MAX = 16


def make_divisible(x, divisor):
    return math.ceil(x / divisor) * divisor


def guess_model_scale(path: str) -> str:
    m = re.search(r"yolo(e-)?[v]?\d+([nslmx])", os.path.splitext(os.path.basename(str(path)))[0])
    return m.group(2) if m else ""


def unified_stem(path: str) -> str:
    stem = os.path.splitext(os.path.basename(str(path)))[0]
    return re.sub(r"(\d+)([nslmx])(.+)?$", r"\1\3", stem)


def load_model_dict(path: str) -> dict:
    """yaml_model_load: a YAML file if it exists, else the built-in topology by unified stem."""
    import copy

    if os.path.isfile(path):
        import yaml

        with open(path) as f:
            d = yaml.safe_load(f)
    else:
        key = unified_stem(path)
        if key not in BUILTIN:
            raise FileNotFoundError(f"model config {path!r} not found (built-in: {sorted(BUILTIN)})")
        d = copy.deepcopy(BUILTIN[key])
    d["scale"] = guess_model_scale(path)
    d["yaml_file"] = str(path)
    return d


@dataclass
class Layer:
    i: int
    f: object          # int or list[int]
    kind: str          # Conv | C2f | SPPF | Upsample | Concat | Detect
    c1: object         # input channels (int, or list for Concat/Detect)
    c2: int            # output channels (Detect: 4*REG_MAX + nc)
    args: dict = field(default_factory=dict)


@dataclass
class Arch:
    layers: list
    save: list
    nc: int
    scale: str
    depth: float
    width: float


def parse_arch(d: dict, ch: int = 3) -> Arch:
    nc = d["nc"]
    scales = d.get("scales")
    depth, width, max_ch = d.get("depth_multiple", 1.0), d.get("width_multiple", 1.0), float("inf")
    scale = d.get("scale") or ""
    if scales:
        if not scale:
            scale = tuple(scales.keys())[0]  # parse_model's "no model scale passed" default
        depth, width, max_ch = scales[scale]
    chs = [ch]
    layers, save = [], []
    for i, (f, n, m, args) in enumerate(d["backbone"] + d["head"]):
        m = m.replace("nn.", "")
        n = max(round(n * depth), 1) if n > 1 else n
        if m in ("Conv", "C2f", "SPPF"):
            c1, c2 = chs[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_ch) * width, 8)
            if m == "Conv":
                k = args[1] if len(args) > 1 else 1
                s = args[2] if len(args) > 2 else 1
                L = Layer(i, f, m, c1, c2, {"k": k, "s": s})
            elif m == "C2f":
                L = Layer(i, f, m, c1, c2, {"n": n, "shortcut": bool(args[1]) if len(args) > 1 else False})
            else:
                L = Layer(i, f, m, c1, c2, {"k": args[1] if len(args) > 1 else 5})
        elif m == "Upsample":
            L = Layer(i, f, m, chs[f], chs[f], {"scale": args[1]})
        elif m == "Concat":
            L = Layer(i, f, m, [chs[x] for x in f], sum(chs[x] for x in f), {})
        elif m == "Detect":
            cin = [chs[x] for x in f]
            c2b = max((16, cin[0] // 4, REG_MAX * 4))
            c3 = max(cin[0], min(nc, 100))
            L = Layer(i, f, m, cin, REG_MAX * 4 + nc, {"nc": nc, "c2": c2b, "c3": c3})
        else:
            raise ValueError(f"module {m!r} is outside the detection hot path")
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(L)
        if i == 0:
            chs = []
        chs.append(L.c2)
    return Arch(layers, sorted(save), nc, scale, depth, width)


def conv_specs(arch: Arch):
    """Every conv of the model in state-dict naming: (prefix, c1, c2, k, s, has_bn_act).
    Detect's final 1x1 convs are plain nn.Conv2d with bias and no BN/act."""
    out = []
    for L in arch.layers:
        p = f"model.{L.i}"
        if L.kind == "Conv":
            out.append((p, L.c1, L.c2, L.args["k"], L.args["s"], True))
        elif L.kind == "C2f":
            c = int(L.c2 * 0.5)
            n = L.args["n"]
            out.append((f"{p}.cv1", L.c1, 2 * c, 1, 1, True))
            for j in range(n):
                out.append((f"{p}.m.{j}.cv1", c, c, 3, 1, True))
                out.append((f"{p}.m.{j}.cv2", c, c, 3, 1, True))
            out.append((f"{p}.cv2", (2 + n) * c, L.c2, 1, 1, True))
        elif L.kind == "SPPF":
            c_ = L.c1 // 2
            out.append((f"{p}.cv1", L.c1, c_, 1, 1, True))
            out.append((f"{p}.cv2", c_ * 4, L.c2, 1, 1, True))
        elif L.kind == "Detect":
            c2b, c3, nc = L.args["c2"], L.args["c3"], L.args["nc"]
            for li, x in enumerate(L.c1):
                out.append((f"{p}.cv2.{li}.0", x, c2b, 3, 1, True))
                out.append((f"{p}.cv2.{li}.1", c2b, c2b, 3, 1, True))
                out.append((f"{p}.cv2.{li}.2", c2b, 4 * REG_MAX, 1, 1, False))
                out.append((f"{p}.cv3.{li}.0", x, c3, 3, 1, True))
                out.append((f"{p}.cv3.{li}.1", c3, c3, 3, 1, True))
                out.append((f"{p}.cv3.{li}.2", c3, nc, 1, 1, False))
    return out


def detect_strides(arch: Arch) -> list:
    """Per-level strides of the Detect inputs (what DetectionModel's stride probe measures,
    tasks.py:409-418): products of conv strides / upsample factors along the graph."""
    st = []
    for L in arch.layers:
        def src(x):
            if x == -1:
                return st[L.i - 1] if L.i else 1
            return st[x]
        if L.kind == "Conv":
            s = src(L.f) * L.args["s"]
        elif L.kind in ("C2f", "SPPF"):
            s = src(L.f)
        elif L.kind == "Upsample":
            s = src(L.f) // L.args["scale"]
        elif L.kind == "Concat":
            s = src(L.f[0])
        else:  # Detect
            return [src(x) for x in L.f]
        st.append(s)
    raise ValueError("no Detect layer")
