"""The shipped gfx950 kernels use no scratch memory and spill no VGPRs.

Read from the code-object metadata of the built libyk.so (CPU only).  A kernel with a private
segment reads and writes per-lane stack memory through the vector memory path on every access:
for the tracker kernels that was 384-1,632 B per thread (dynamically indexed local arrays and a
non-inlined helper taking pointers to locals); for the 8-wave conv_wide tiles it was VGPR spills,
which the autotuner could pick.  SGPR spills land in VGPR lanes (v_writelane), not in memory, and
are reported, not failed."""
import pytest

import co_helpers as CO
from conftest import pkg


@pytest.fixture(scope="module")
def kernels():
    if not CO.available():
        pytest.skip("ROCm LLVM tools missing")
    lib = pkg()._lib.LIB_PATH
    ks = CO.kernels(lib)
    assert len(ks) > 100, len(ks)  # every HIP source's bundle was read
    return ks


def test_no_kernel_uses_scratch(kernels):
    bad = [k for k in kernels if k["scratch"] > 0]
    names = CO.demangle([k["name"] for k in bad])
    assert not bad, [(n[:100], k["scratch"]) for n, k in zip(names, bad)]


def test_no_kernel_spills_vgprs(kernels):
    bad = [k for k in kernels if k["vgpr_spill"] > 0]
    names = CO.demangle([k["name"] for k in bad])
    assert not bad, [(n[:100], k["vgpr_spill"]) for n, k in zip(names, bad)]


def test_every_source_is_in_the_library(kernels):
    names = " ".join(CO.demangle([k["name"] for k in kernels]))
    for k in ("conv_fast_kernel", "nms_kernel", "detect_kernel", "assoc_kernel", "tracks_kernel", "bt_step_kernel",
              "lk_kernel", "gmc_kernel"):
        assert k in names, k


def test_sgpr_spills_reported(kernels):
    """SGPR spills go to VGPR lanes, not memory; list them (and keep them bounded)."""
    sp = [(n, k["sgpr_spill"]) for n, k in zip(CO.demangle([k["name"] for k in kernels]), kernels) if k["sgpr_spill"]]
    for n, c in sp:
        print("SGPR_SPILL", c, n[:100])
    assert all(c <= 128 for _, c in sp)
