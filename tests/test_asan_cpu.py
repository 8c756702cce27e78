"""AddressSanitizer + UBSan build of the C ABI's host-side parsers (VERDICT r5 hygiene item).

yk_host.cpp (the detector-program validation yk_model_create runs first, and yk_model_load's
engine-file reader) and program.cpp (yk_program_build: the state dict -> program builder) take
input from outside the library.  They contain no HIP code, so they are built here on the CPU with
-fsanitize=address,undefined together with tests/asan/host_fuzz.cpp and fed real engines and
state dicts (which must be accepted) and corrupted ones (truncations, flipped bytes, extreme
header / descriptor / op / buffer fields, garbage, missing or mis-shaped tensors, non-finite
weights, bad sizes), which must be rejected or accepted without a sanitizer report."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO, pkg

CLANG = "/opt/rocm/lib/llvm/bin/clang++"
CSRC = os.path.join(REPO, "yolo---small-target-recognition---kalman-trajectory-prediction_amd", "csrc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    cxx = CLANG if os.path.exists(CLANG) else shutil.which("clang++")
    if cxx is None:
        pytest.skip("clang++ missing (program.cpp needs _Float16 on the host)")
    out = str(tmp_path_factory.mktemp("asan") / "host_fuzz")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"), "-I", CSRC,
           os.path.join(CSRC, "yk_host.cpp"), os.path.join(CSRC, "program.cpp"),
           os.path.join(REPO, "tests", "asan", "host_fuzz.cpp"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return out


def _run(args, timeout=600):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    return r


def _engine(tmp_path, scale, dtype, hw=(512, 640), imgsz=640, max_batch=2, plan=False):
    import importlib

    P = pkg()
    A = importlib.import_module(P.__name__ + ".arch")
    M = importlib.import_module(P.__name__ + ".model")
    W = importlib.import_module(P.__name__ + ".weights")
    ar = A.parse_arch(A.load_model_dict(f"yolov8{scale}-small.yaml"))
    prog = M.Program(ar, W.synthetic_state_dict(ar, 0), hw[0], hw[1], imgsz, max_batch, dtype)
    path = str(tmp_path / f"{scale}_{dtype}_{hw[1]}x{hw[0]}.yke")
    pl = [[3, 2, 4] if op.kind == M.YK_K_CONV else [-1, 0, 0] for op in prog.ops] if plan else None
    prog.export_engine(path, pl, max_batch if plan else 0)
    return path


@pytest.mark.parametrize("scale,dtype,hw,imgsz", [("n", "fp32", (512, 640), 640), ("s", "bf16", (1080, 1920), 640),
                                                  ("n", "fp8", (1024, 1280), 1280), ("n", "fp16", (375, 1242), 640)])
def test_real_engines_accepted_and_corrupt_ones_rejected_cleanly(harness, tmp_path, scale, dtype, hw, imgsz):
    path = _engine(tmp_path, scale, dtype, hw, imgsz, plan=True)
    r = _run([harness, "engine", path])
    assert r.returncode == 0, r.stderr
    r = _run([harness, "engine-fuzz", path, "7", "400"])
    assert r.returncode == 0, r.stderr
    line = r.stdout.strip().splitlines()[-1]
    print(line)
    acc = int(line.split("accepted=")[1].split()[0])
    assert acc < 400  # the corruptions are seen


def test_program_builder_under_sanitizers(harness, tmp_path):
    import importlib

    P = pkg()
    A = importlib.import_module(P.__name__ + ".arch")
    W = importlib.import_module(P.__name__ + ".weights")
    ar = A.parse_arch(A.load_model_dict("yolov8n-small.yaml"))
    wpath = str(tmp_path / "n.ykw")
    W.save_raw(wpath, W.synthetic_state_dict(ar, 0))
    r = _run([harness, "program", wpath, "150"], timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    print(r.stdout.strip())
    assert "scale=n" in r.stdout
