"""Write a structurally faithful ultralytics-style checkpoint without ultralytics: a pickled
module tree whose classes carry ultralytics' qualified names (ultralytics.nn.tasks.DetectionModel,
ultralytics.nn.modules.{conv,block,head}.*) over real torch.nn Conv2d / BatchNorm2d / SiLU /
Sequential / ModuleList leaves, fp16 weights, the parsed YAML on model.yaml and the
strip_optimizer keys (utils/torch_utils.py:714-773).  Test fixture generator only."""
import sys
import types

import torch
import torch.nn as nn

_FAKE = {
    "ultralytics.nn.tasks": ["DetectionModel"],
    "ultralytics.nn.modules.conv": ["Conv", "Concat"],
    "ultralytics.nn.modules.block": ["C2f", "Bottleneck", "SPPF", "DFL"],
    "ultralytics.nn.modules.head": ["Detect"],
    "ultralytics.utils": ["IterableSimpleNamespace"],
}


def _fake_classes():
    out = {}
    for mod, names in _FAKE.items():
        parts = mod.split(".")
        for i in range(1, len(parts) + 1):
            sys.modules.setdefault(".".join(parts[:i]), types.ModuleType(".".join(parts[:i])))
        m = sys.modules[mod]
        for n in names:
            if not hasattr(m, n):
                base = (object,) if n == "IterableSimpleNamespace" else (nn.Module,)
                setattr(m, n, type(n, base, {"__module__": mod, "__qualname__": n}))
            out[n] = getattr(m, n)
    return out


def _leaf(parent_path, name, shape_params):
    """A torch.nn leaf for a parameter group: conv / bn / plain conv with bias."""
    w = shape_params.get("weight")
    if name == "bn":
        bn = nn.BatchNorm2d(w.shape[0], eps=1e-3, momentum=0.03)
        return bn
    conv = nn.Conv2d(w.shape[1], w.shape[0], w.shape[2], bias="bias" in shape_params)
    return conv


def build_module_tree(ar, sd):
    C = _fake_classes()
    kinds = {f"model.{Ly.i}": Ly.kind for Ly in ar.layers}
    root = C["DetectionModel"]()
    seq = nn.Sequential()
    root.add_module("model", seq)
    groups = {}
    for k, v in sd.items():
        path, leafname = k.rsplit(".", 1)
        groups.setdefault(path, {})[leafname] = v
    for Ly in ar.layers:
        cls = {"Conv": "Conv", "C2f": "C2f", "SPPF": "SPPF", "Concat": "Concat", "Detect": "Detect"}.get(Ly.kind)
        mod = nn.Upsample(scale_factor=2, mode="nearest") if Ly.kind == "Upsample" else C[cls]()
        seq.add_module(str(Ly.i), mod)
    for path in sorted(groups, key=lambda p: [int(x) if x.isdigit() else x for x in p.split(".")]):
        parts = path.split(".")
        cur = root
        for j, part in enumerate(parts):
            sub = cur._modules.get(part)
            if sub is None:
                last = j == len(parts) - 1
                if last:
                    sub = _leaf(".".join(parts[:j]), part, groups[path])
                elif part == "m" and kinds.get(".".join(parts[:2])) in ("C2f",):
                    sub = nn.ModuleList()
                elif part in ("cv2", "cv3") and kinds.get(".".join(parts[:2])) == "Detect":
                    sub = nn.ModuleList()
                elif kinds.get(".".join(parts[:2])) == "Detect" and parts[j - 1] in ("cv2", "cv3"):
                    sub = nn.Sequential()
                elif part == "dfl":
                    sub = C["DFL"]()
                elif parts[j - 1] == "m" and part.isdigit():
                    sub = C["Bottleneck"]()
                else:
                    sub = C["Conv"]()
                if part.isdigit() and isinstance(cur, nn.ModuleList):
                    cur.append(sub)
                else:
                    cur.add_module(part, sub)
            cur = sub
        for name, t in groups[path].items():
            if name in ("weight", "bias"):
                cur._parameters[name] = nn.Parameter(t.clone(), requires_grad=False)
            else:
                cur._buffers[name] = t.clone()
        if isinstance(cur, nn.Conv2d) or isinstance(cur, nn.BatchNorm2d):
            pass
    return root


def write_checkpoint(path, ar, yaml_dict, sd, half=True):
    """The stand-in ultralytics modules live in sys.modules only while the file is written, so a
    later ``from ultralytics import YOLO`` (the compat package) is not shadowed by them."""
    before = set(sys.modules)
    try:
        return _write_checkpoint(path, ar, yaml_dict, sd, half)
    finally:
        for k in set(sys.modules) - before:
            if k == "ultralytics" or k.startswith("ultralytics."):
                del sys.modules[k]


def _write_checkpoint(path, ar, yaml_dict, sd, half):
    C = _fake_classes()
    model = build_module_tree(ar, sd)
    if half:
        model.half()
    model.yaml = dict(yaml_dict)
    model.stride = torch.tensor([4.0, 8.0, 16.0, 32.0])
    model.names = {0: "aircraft"}
    args = C["IterableSimpleNamespace"]()
    args.__dict__.update({"imgsz": 640, "seed": 0})
    model.args = args
    ckpt = {"date": "2025-01-01T00:00:00", "version": "8.3.193", "license": "AGPL-3.0", "docs": "",
            "epoch": -1, "best_fitness": None, "model": model, "ema": None, "updates": None, "optimizer": None,
            "train_args": {"imgsz": 640, "seed": 0, "model": "yolov8-small.yaml"}}
    torch.save(ckpt, path)
    return model
