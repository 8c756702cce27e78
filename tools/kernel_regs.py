#!/usr/bin/env python3
"""Register / LDS / scratch use of the gfx950 kernels in a built object (the code-object notes of
its offload bundle) and the waves per SIMD that allows (512 unified VGPR + AGPR registers per
lane, allocated in granules of 8).

usage: kernel_regs.py OBJECT.o [substring ...]"""
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(obj):
    with tempfile.TemporaryDirectory() as d:
        fb, co = f"{d}/fatbin", f"{d}/k.co"
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, f"{d}/junk"], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout


def main():
    obj, subs = sys.argv[1], sys.argv[2:]
    for b in notes(obj).split("  - .agpr_count:")[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", b)
            return m.group(1) if m else "0"
        agpr = int(b.split("\n", 1)[0].strip())
        name = subprocess.run(["c++filt", g("name")], capture_output=True, text=True).stdout.strip()
        name = name.replace("void ", "").replace("yk::det::", "").replace("yk::trk::", "")
        if subs and not any(s in name for s in subs):
            continue
        v = int(g("vgpr_count"))
        tot = ((v + 7) // 8) * 8 + ((agpr + 7) // 8) * 8
        print(f"{name[:64]:64s} vgpr {v:3d} agpr {agpr:3d} sgpr {g('sgpr_count'):>3s} lds {g('group_segment_fixed_size'):>6s} "
              f"scratch {g('private_segment_fixed_size'):>4s} waves/SIMD {min(8, 512 // max(tot, 1))}")


if __name__ == "__main__":
    main()
