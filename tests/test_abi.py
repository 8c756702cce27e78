"""libyk.so loads on a CPU-only host and exports every function include/yk.h declares;
the ctypes mirrors of the ABI structs have the C sizes.  No compute call is made."""
import ctypes
import os
import re

import pytest

from conftest import REPO, pkg

HEADER = os.path.join(REPO, "include", "yk.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s+\*?(yk_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for n in ("yk_ctx_create", "yk_tracker_create", "yk_tracker_step", "yk_tracker_download", "yk_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from importlib import import_module

    lib_mod = import_module(pkg().__name__ + "._lib")
    lib = lib_mod.lib()  # loads libyk.so (raises if missing)
    for n in declared_functions():
        assert hasattr(lib, n), f"libyk.so does not export {n}"
    # the python binding covers every declared function too
    assert set(declared_functions()) <= set(lib_mod.exported_symbols())


def test_struct_sizes_match_python_mirrors():
    from importlib import import_module

    L = import_module(pkg().__name__ + "._lib")
    lib = L.lib()
    assert lib.yk_struct_size(0) == ctypes.sizeof(L.TrackerCfg)
    assert lib.yk_struct_size(1) == L.STATS_DTYPE.itemsize
    assert lib.yk_struct_size(2) == L.TRACK_OUT_DTYPE.itemsize
    assert lib.yk_struct_size(3) == L.TRACK_STATE_DTYPE.itemsize
    assert lib.yk_struct_size(7) == ctypes.sizeof(L.BtCfg)
    assert lib.yk_struct_size(8) == L.MOTION_DTYPE.itemsize
    assert lib.yk_struct_size(9) == L.GMD_STATS_DTYPE.itemsize
    assert lib.yk_struct_size(10) == ctypes.sizeof(L.Tensor)
    assert lib.yk_struct_size(99) == -1


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg().YKError):
        pkg().EnhancedMultiTargetTracker(150, 1, 0.1)
