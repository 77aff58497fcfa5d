"""Register / scratch / LDS budgets of the built gfx950 kernels, read from the code objects' metadata (no GPU).

The 8-phase GEMM schedule assumes every production instantiation runs spill-free: a kernel with a private
(scratch) segment puts scratch loads and stores -- and the ``s_waitcnt vmcnt(0)`` hipcc emits around them -- inside
the counted-``vmcnt`` main loop, which both drains the LDS-DMA pipeline and, in round 5, preceded a GPU memory-
aperture fault in a diagnostic build that spilled (docs/DESIGN.md §2).  ``check_built()`` extracts the gfx950 code
object from each built GEMM object (``build/gemm*.hip.o``: offload bundle in ``.hip_fatbin``), parses the AMDGPU
metadata notes and returns every budget violation; ``tests/test_kernel_resources_cpu.py`` runs it in the CPU suite.

    python -m dllm.utils.kernel_resources            # table of the GEMM kernels + violations
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(PKG, "build")

# production GEMM families: (mangled-name prefix, VGPR+AGPR budget per lane, LDS bytes the schedule assumes or None)
#   8-phase 256x256 (+ grouped pair, 224-row): 512 threads, __launch_bounds__(512, 2) -> 2 waves per SIMD -> 256
#   registers of the unified 512-entry file; 8 x 16 KiB half-tile slots = 128 KiB of LDS (+ 8 KiB: the epilogue-operand
#   prefetch sink of the fused-optimizer / ReLU-dgrad / SwiGLU-dgrad instantiations)
#   256x128 ping-pong: 2 blocks of 4 waves per CU -> 2 waves per SIMD -> 256; 80 KiB each (two fit in 160 KiB)
FAMILIES = (
    ("_ZN4dllm13gemm_bf16_8phI", 256, (131072, 139264)),
    ("_ZN4dllm18gemm_bf16_8ph_pairI", 256, (131072, 139264)),
    ("_ZN4dllm18gemm_bf16_8ph_m224I", 256, (131072,)),
    ("_ZN4dllm12gemm_bf16_ppI", 256, (81920,)),
    ("_ZN4dllm13gemm_bf16_256I", 256, None),
    ("_ZN4dllm12gemm_f32_256I", 256, None),
    ("_ZN4dllm12gemm_f32_128I", 256, None),
)
LDS_MAX = 160 * 1024


def _tool(name: str) -> str:
    p = os.path.join(LLVM, name)
    if not os.path.exists(p):
        raise RuntimeError(f"{p} not found (ROCm LLVM tools)")
    return p


def device_code_object(obj: str, out: str) -> str:
    """The gfx950 code object of a host object built by hipcc (its ``.hip_fatbin`` offload bundle)."""
    fat = out + ".fat"
    subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj, os.devnull], check=True,
                   capture_output=True)
    subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--targets={TARGET}",
                    f"--input={fat}", f"--output={out}"], check=True, capture_output=True)
    os.remove(fat)
    return out


def kernels(code_object: str) -> list[dict]:
    """Per-kernel resources from the AMDGPU metadata notes of a gfx950 code object."""
    notes = subprocess.run([_tool("llvm-readelf"), "--notes", code_object], check=True, capture_output=True,
                           text=True).stdout
    out = []
    for blk in notes.split("  - .agpr_count:")[1:]:
        get = lambda k: re.search(rf"\.{k}:\s+(\S+)", blk)  # noqa: E731
        name = get("name")
        if name is None or get("vgpr_count") is None:
            continue
        out.append({"name": name.group(1), "agpr": int(blk.split("\n", 1)[0].strip()),
                    "vgpr": int(get("vgpr_count").group(1)), "sgpr": int(get("sgpr_count").group(1)),
                    "scratch": int(get("private_segment_fixed_size").group(1)),
                    "lds": int(get("group_segment_fixed_size").group(1))})
    return out


def violations(recs: list[dict], families=FAMILIES) -> list[str]:
    """Budget violations of the production GEMM kernels among ``recs`` (all kernels: no scratch at all)."""
    bad = []
    for r in recs:
        if r["scratch"] > 0:
            bad.append(f"{r['name']}: {r['scratch']} B of scratch (register spill / private array)")
        if r["lds"] > LDS_MAX:
            bad.append(f"{r['name']}: {r['lds']} B of LDS > {LDS_MAX}")
        for prefix, regs, lds in families:
            if r["name"].startswith(prefix):
                # the unified register file: arch VGPRs (allocated in granules of 8) + AGPRs per lane
                used = -(-r["vgpr"] // 8) * 8 + r["agpr"]
                if used > regs:
                    bad.append(f"{r['name']}: {r['vgpr']} VGPR + {r['agpr']} AGPR > {regs}")
                if lds is not None and r["lds"] not in lds:
                    bad.append(f"{r['name']}: {r['lds']} B of LDS, the schedule assumes one of {lds}")
    return bad


def built_objects(build_dir: str = BUILD) -> list[str]:
    return sorted(os.path.join(build_dir, f) for f in os.listdir(build_dir)
                  if f.startswith("gemm") and f.endswith(".hip.o"))


def check_built(build_dir: str = BUILD) -> tuple[list[dict], list[str]]:
    """(every kernel of the built GEMM objects, the budget violations among them)."""
    recs = []
    with tempfile.TemporaryDirectory() as d:
        for obj in built_objects(build_dir):
            co = device_code_object(obj, os.path.join(d, os.path.basename(obj) + ".co"))
            for r in kernels(co):
                r["object"] = os.path.basename(obj)
                recs.append(r)
    return recs, violations(recs)


def main() -> int:
    import subprocess as sp

    recs, bad = check_built()
    dem = sp.run(["c++filt"], input="\n".join(r["name"] for r in recs), capture_output=True, text=True).stdout.split("\n")
    for r, d in zip(recs, dem):
        if any(r["name"].startswith(p) for p, _, _ in FAMILIES):
            print(f"vgpr {r['vgpr']:>4} agpr {r['agpr']:>3} sgpr {r['sgpr']:>3} scratch {r['scratch']:>5} "
                  f"lds {r['lds']:>6}  {d[:140]}")
    print(f"{len(recs)} kernels, {len(bad)} violations")
    for b in bad:
        print("VIOLATION", b)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
