"""Kernel descriptors of the gfx950 code objects inside libyk.so (no GPU needed).

The library's .hip_fatbin section holds one clang offload bundle per HIP source (tracker,
detector, bytetrack, gmd); each gfx950 code object's AMDGPU metadata note lists every kernel with
its register counts, spills and private (scratch) segment size."""
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def available() -> bool:
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf"))


def kernels(lib_path: str) -> list[dict]:
    """[{name, vgpr, agpr, sgpr, sgpr_spill, vgpr_spill, scratch, lds}] of every gfx950 kernel."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib_path, os.path.join(d, "junk")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for i in range(len(starts) - 1):
            part = os.path.join(d, f"b{i}")
            with open(part, "wb") as f:
                f.write(data[starts[i]:starts[i + 1]])
            co = os.path.join(d, f"k{i}.co")
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                           capture_output=True)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                                   check=True).stdout
            for b in notes.split("  - .agpr_count:")[1:]:
                def g(k, blk=b):
                    m = re.search(r"\." + k + r":\s+(\S+)", blk)
                    return m.group(1) if m else "0"
                out.append({"name": g("name"), "agpr": int(b.split("\n", 1)[0].strip()), "vgpr": int(g("vgpr_count")),
                            "sgpr": int(g("sgpr_count")), "sgpr_spill": int(g("sgpr_spill_count")),
                            "vgpr_spill": int(g("vgpr_spill_count")),
                            "scratch": int(g("private_segment_fixed_size")),
                            "lds": int(g("group_segment_fixed_size"))})
    return out


def demangle(names: list[str]) -> list[str]:
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names
