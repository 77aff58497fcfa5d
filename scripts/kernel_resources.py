"""Per-kernel register / scratch / LDS usage of a GEMM translation unit (device-only gfx950 compile + the
code object's metadata notes): catches spills (private segment > 0) and VGPR blow-ups without a GPU.

    python scripts/kernel_resources.py [gemm_tn.hip] [--filter SUBSTR] [-D NAME=VALUE ...]
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed-llm-code-samples_amd", "csrc")
LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?", default="gemm_tn.hip")
    ap.add_argument("--filter", default="gemm_bf16_8ph")
    ap.add_argument("-D", action="append", default=[], help="extra preprocessor define (NAME=VALUE)")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        obj = os.path.join(d, "k.o")
        subprocess.run(["hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output", "-c",
                        *[f"-D{d}" for d in a.D], "-I", CSRC, os.path.join(CSRC, a.src), "-o", obj], check=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", obj], capture_output=True,
                               text=True, check=True).stdout
        dem = subprocess.run(["c++filt"], input=notes, capture_output=True, text=True).stdout
    # metadata is YAML-ish: one "- .args:" block per kernel
    blocks = dem.split("  - .agpr_count:")
    for b in blocks[1:]:
        name = re.search(r"\.name:\s+(.*)", b)
        if not name or a.filter not in name.group(1):
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", b) or [None, "?"])[1]  # noqa: E731
        agpr = b.split("\n", 1)[0].strip()
        print(f"vgpr {get('vgpr_count'):>4} agpr {agpr:>4} sgpr {get('sgpr_count'):>3} "
              f"scratch {get('private_segment_fixed_size'):>5} lds {get('group_segment_fixed_size'):>6}  "
              f"{name.group(1)[:150]}")


if __name__ == "__main__":
    main()
