"""Audit a GEMM kernel's gfx950 assembly for pipeline-draining waits (no GPU needed).

    python scripts/asm_audit.py gemm_tn.hip gemm_bf16_pp ILi2ELi5E [--dump]

Compiles the translation unit device-only to assembly, picks the kernels whose mangled name contains every
filter substring, and prints per kernel: VGPR / scratch, the number of MFMAs, LDS-DMA and barriers, and every
`s_waitcnt` that waits for vmcnt inside a loop block (a `vmcnt(0)` there drains the LDS-DMA pipeline: the
§5 'Pipelining across barriers' trap).  --dump prints the loop blocks' control/wait skeleton.
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed-llm-code-samples_amd", "csrc")


def kernels(asm: str):
    for m in re.finditer(r"^(_Z\S+):\s*;", asm, re.M):
        name = m.group(1)
        end = asm.find(".Lfunc_end", m.end())
        yield name, asm[m.end():end]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("filters", nargs="+")
    ap.add_argument("--dump", action="store_true")
    ap.add_argument("-D", action="append", default=[])
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        *[f"-D{x}" for x in a.D], "-I", CSRC, os.path.join(CSRC, a.src), "-o", out], check=True,
                       stderr=subprocess.DEVNULL)
        asm = open(out).read()
    for name, body in kernels(asm):
        if not all(f in name for f in a.filters):
            continue
        vg = re.search(rf"{re.escape(name)}\.num_vgpr, (\d+)", asm)
        sc = re.search(rf"{re.escape(name)}\.private_seg_size, (\d+)", asm)
        lines = [l.strip() for l in body.split("\n")]
        n_mfma = sum(l.startswith("v_mfma") for l in lines)
        n_glds = sum("global_load_lds" in l for l in lines)
        n_bar = sum(l.startswith("s_barrier") for l in lines)
        print(f"{name}: vgpr {vg.group(1) if vg else '?'} scratch {sc.group(1) if sc else '?'} "
              f"mfma {n_mfma} glds {n_glds} barriers {n_bar}")
        # loop blocks: labels that are targets of a backward branch
        labels = {l[:-1]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\S+:$", l)}
        loops = []
        for i, l in enumerate(lines):
            m = re.match(r"^s_cbranch_\w+\s+(\.LBB\S+)|^s_branch\s+(\.LBB\S+)", l)
            if m:
                t = m.group(1) or m.group(2)
                if t in labels and labels[t] < i:
                    loops.append((labels[t], i))
        for (s, e) in loops:
            waits = [lines[k] for k in range(s, e + 1) if lines[k].startswith("s_waitcnt") and "vmcnt" in lines[k]]
            mf = sum(lines[k].startswith("v_mfma") for k in range(s, e + 1))
            print(f"  loop {lines[s]} .. {e - s} lines, {mf} mfma, vmcnt waits: {waits}")
            if a.dump:
                for k in range(s, e + 1):
                    l = lines[k]
                    if l.startswith(("s_waitcnt", "s_barrier", ".LBB", "s_cbranch", "s_branch", "s_setprio")) or \
                            "global_load_lds" in l:
                        print("     ", l[:90])


if __name__ == "__main__":
    main()
