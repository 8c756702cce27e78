"""Ultralytics ``*.pt`` checkpoints -> (model YAML dict, state dict), without ultralytics and
without executing anything from the file.

Reference format (utils/torch_utils.py:714-773 strip_optimizer, nn/tasks.py:1404-1521
torch_safe_load / load_checkpoint): ``torch.save`` of a dict whose ``'model'`` (or ``'ema'``)
entry is a pickled ``ultralytics.nn.tasks.DetectionModel`` in fp16, carrying its parsed YAML
(``model.yaml``, incl. ``'scale'``) and ``train_args``.  The reference unpickles it with the
real ultralytics classes (or its SafeUnpickler, which still runs pickle's REDUCE on torch
callables).

Here the file goes through ``torch.load(weights_only=True)`` only.  Every global the pickle
names that is not on torch's weights-only allowlist (the ultralytics module classes, torch.nn
module classes, IterableSimpleNamespace, loss classes, ...) is replaced by an inert stub class
with the same qualified name: NEWOBJ creates a bare stub, BUILD only fills its ``__dict__``,
REDUCE on a stub constructs an empty stub (its ``__init__`` ignores its arguments).  So no
callable from the file runs; tensors are rebuilt by torch's own allowlisted rebuild functions.
The module tree is then walked through the stubs' ``_modules`` / ``_parameters`` / ``_buffers``
dicts (nn.Module's pickled state) to produce the ``model.{i}.*`` state dict that
weights.fused_convs / model.Program pack for the kernels, in float32 (load_checkpoint's
``.float()``, tasks.py:1490).
"""
from __future__ import annotations

from collections import OrderedDict

import torch


def _stub(full_name: str):
    module, _, qual = full_name.rpartition(".")

    def __init__(self, *args, **kwargs):  # REDUCE on a stub: an inert empty instance
        pass

    def __call__(self, *args, **kwargs):
        return None

    cls = type(qual, (), {"__init__": __init__, "__call__": __call__, "__module__": module, "__qualname__": qual,
                          "__doc__": f"inert stand-in for {full_name} (checkpoint.py)"})
    return (cls, full_name)


def load_raw(path: str) -> dict:
    """The checkpoint dict with every non-allowlisted global stubbed (weights_only load)."""
    names = torch.serialization.get_unsafe_globals_in_checkpoint(path)
    stubs = [_stub(n) for n in names]
    with torch.serialization.safe_globals(stubs):
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(ckpt, dict):  # torch.save(model) instead of a checkpoint dict (tasks.py:1451-1457)
        ckpt = {"model": getattr(ckpt, "model", ckpt)}
    return ckpt


def _attrs(obj) -> dict:
    return obj.__dict__ if hasattr(obj, "__dict__") else {}


def module_state_dict(mod, prefix: str = "") -> "OrderedDict[str, torch.Tensor]":
    """nn.Module.state_dict() restated over the pickled module state: parameters and
    persistent buffers, depth first in registration order."""
    out = OrderedDict()
    d = _attrs(mod)
    for k, v in (d.get("_parameters") or {}).items():
        if v is not None:
            out[prefix + k] = v.detach() if isinstance(v, torch.Tensor) else v
    skip = set(d.get("_non_persistent_buffers_set") or ())
    for k, v in (d.get("_buffers") or {}).items():
        if v is not None and k not in skip:
            out[prefix + k] = v
    for k, m in (d.get("_modules") or {}).items():
        if m is not None:
            out.update(module_state_dict(m, prefix + k + "."))
    return out


def load_checkpoint(path: str):
    """(yaml dict, float32 state dict, checkpoint metadata) of an ultralytics detection checkpoint."""
    ckpt = load_raw(path)
    model = ckpt.get("ema") or ckpt.get("model")
    if model is None:
        raise ValueError(f"{path}: no 'model' / 'ema' entry (not an ultralytics checkpoint)")
    attrs = _attrs(model)
    y = attrs.get("yaml")
    if not isinstance(y, dict) or "backbone" not in y or "head" not in y:
        raise ValueError(f"{path}: the pickled model carries no parsed model YAML (model.yaml)")
    sd = OrderedDict((k, v.float() if torch.is_tensor(v) and v.is_floating_point() else v)
                     for k, v in module_state_dict(model).items())
    if not any(k.startswith("model.") for k in sd):
        raise ValueError(f"{path}: no 'model.*' tensors found in the pickled module tree")
    meta = {k: ckpt.get(k) for k in ("epoch", "date", "version", "train_args") if k in ckpt}
    return dict(y), sd, meta
