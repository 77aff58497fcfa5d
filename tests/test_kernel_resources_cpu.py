"""Register / scratch / LDS budgets of every built GEMM kernel, on the CPU: the gfx950 code
objects' metadata (utils/kernel_resources.py).  A spill (private segment > 0) puts scratch traffic -- and hipcc's
``vmcnt(0)`` around it -- inside the counted-vmcnt main loop; the round-5 aperture fault came from a spilling build."""
import os
import subprocess
import tempfile

import pytest

from dllm import _build
from dllm.utils import kernel_resources as kr

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(kr.LLVM, "llvm-readelf")), reason="no ROCm LLVM tools")


@pytest.fixture(scope="module")
def built():
    _build.build()   # incremental: a no-op when the in-tree objects are current
    return kr.check_built()


def test_every_gemm_kernel_within_budget(built):
    recs, bad = built
    fams = [r for r in recs if any(r["name"].startswith(p) for p, _, _ in kr.FAMILIES)]
    # the 8-phase family alone has > 100 instantiations over the three layout units
    assert len([r for r in fams if r["name"].startswith("_ZN4dllm13gemm_bf16_8phI")]) > 100, len(fams)
    assert not bad, "\n".join(bad)


def test_flagship_kernels_present(built):
    """The headline step's kernels are among the checked ones: persistent NT ReLU forward (mask), NN store with the
    transposed copy, NT ReLU dgrad, and the NN-T fused split-master SGD weight gradient."""
    names = {r["name"] for r in built[0]}
    for frag in ("gemm_bf16_8phILi0ELi1EtLb1ELi1ELi8ELb1E",      # NT, EPI_ACT, bf16, ReLU, persistent
                 "gemm_bf16_8phILi1ELi11EtLb1ELin1ELi8ELb1E",    # NN, EPI_STORE_DT, persistent
                 "gemm_bf16_8phILi0ELi2EtLb1ELi1ELi8ELb1E",      # NT, EPI_DACT, ReLU, persistent
                 "gemm_bf16_8phILi1ELi9EfLb1ELin1ELi8ELb1E"):    # NN, EPI_SGDS_T, persistent
        assert any(frag in n for n in names), frag


SPILL = r"""
#include <hip/hip_runtime.h>
__global__ void spills(float* out, const int* idx) {
  float a[256];   // indexed at run time: the array lives in scratch (private segment)
  for (int i = 0; i < 256; ++i) a[i] = out[threadIdx.x + i];
  out[threadIdx.x] = a[idx[threadIdx.x] & 255];
}
"""


def test_checker_flags_a_spilling_kernel():
    """The checker is not vacuous: a deliberately spilling kernel is reported."""
    with tempfile.TemporaryDirectory() as d:
        src, obj = os.path.join(d, "spill.hip"), os.path.join(d, "spill.o")
        with open(src, "w") as f:
            f.write(SPILL)
        subprocess.run([_build._hipcc(), "-O3", "--offload-arch=gfx950", "-c", src, "-o", obj], check=True,
                       capture_output=True)
        recs = kr.kernels(kr.device_code_object(obj, os.path.join(d, "spill.co")))
    (r,) = [r for r in recs if "spills" in r["name"]]
    assert r["scratch"] >= 1024
    bad = kr.violations(recs)
    assert any("scratch" in b and "spills" in b for b in bad), bad
    # and a register budget breach of a production family is reported too
    fake = dict(r, name="_ZN4dllm13gemm_bf16_8phIfake", scratch=0, vgpr=264, agpr=0, lds=131072)
    assert any("VGPR" in b for b in kr.violations([fake]))
