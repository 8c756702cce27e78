"""libyk.so loads on a CPU-only host and exports every function include/yk.h declares;
the ctypes mirrors of the ABI structs have the C sizes.  No compute call is made."""
import ctypes
import os
import re

import pytest

from conftest import REPO, pkg

HEADER = os.path.join(REPO, "include", "yk.h")
DIAG_HEADER = os.path.join(REPO, "include", "yk_diag.h")


def declared_functions(path=HEADER):
    src = open(path).read()
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
    for n in declared_functions() + declared_functions(DIAG_HEADER):
        assert hasattr(lib, n), f"libyk.so does not export {n}"
    # the python binding covers every declared function too
    assert set(declared_functions()) <= set(lib_mod.exported_symbols())


def test_diagnostics_stay_out_of_the_product_header():
    """yk_gmd_debug_* (stream-order copies of the motion detector's internals for parity tools)
    live in yk_diag.h, not in the boundary header (VERDICT r4 hygiene)."""
    diag = declared_functions(DIAG_HEADER)
    assert {"yk_gmd_debug_buffers", "yk_gmd_debug_pyramids"} <= set(diag)
    assert not set(diag) & set(declared_functions())


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
    assert lib.yk_struct_size(11) == L.TRACK_EVENT_DTYPE.itemsize
    assert lib.yk_struct_size(99) == -1


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg().YKError):
        pkg().EnhancedMultiTargetTracker(150, 1, 0.1)


def test_c_host_abi_check_passes_against_this_library(tmp_path):
    """The header-inline yk_abi_check() (version + every struct size, compiled with the host's
    view of the structs) returns YK_OK against the built libyk.so; a host compiled with a
    different YK_ABI_VERSION gets YK_ERR_STATE.  Only yk_abi_version / yk_struct_size are called
    (no GPU)."""
    import shutil
    import subprocess

    if shutil.which("gcc") is None:
        pytest.skip("gcc missing")
    lib_dir = os.path.dirname(pkg()._lib.LIB_PATH)
    src = tmp_path / "abi.c"
    src.write_text('#include <stdio.h>\n#include "yk.h"\nint main(void) { printf("%d\\n", yk_abi_check()); return 0; }\n')
    out = {}
    for tag, extra in (("same", []), ("other", ["-DYK_ABI_OVERRIDE"])):
        exe = tmp_path / f"abi_{tag}"
        cflags = ["-I", os.path.join(REPO, "include")]
        if extra:  # a host built against another header version
            hdr = tmp_path / "old" / "yk.h"
            hdr.parent.mkdir()
            hdr.write_text(open(HEADER).read().replace("#define YK_ABI_VERSION 3", "#define YK_ABI_VERSION 2"))
            cflags = ["-I", str(hdr.parent)]
        subprocess.run(["gcc", "-std=c11", *cflags, str(src), "-L", lib_dir, "-l:libyk.so",
                        f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True, capture_output=True)
        r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        out[tag] = int(r.stdout.strip())
    assert out == {"same": 0, "other": 4}, out


def test_round5_entry_points_refuse_bad_arguments_without_a_device():
    """yk_upload_pinned_async / yk_tracker_download_async check their arguments before any device
    call: NULL pointers and sizes that are not multiples of 16 come back as YK_ERR_ARG with a
    message (callable on this CPU-only host)."""
    P = pkg()
    L = P._lib
    lib = L.lib()
    buf = ctypes.create_string_buffer(64)
    for args in ((None, None, 16, None), (ctypes.addressof(buf), None, 16, None),
                 (ctypes.addressof(buf), ctypes.addressof(buf), 15, None)):
        rc = lib.yk_upload_pinned_async(*args)
        assert rc != 0
        assert b"yk_upload_pinned_async" in ctypes.cast(lib.yk_last_error(), ctypes.c_char_p).value
    rc = lib.yk_tracker_download_async(None, None, None, None, 0, None)
    assert rc != 0
    assert b"yk_tracker_download_async" in ctypes.cast(lib.yk_last_error(), ctypes.c_char_p).value
