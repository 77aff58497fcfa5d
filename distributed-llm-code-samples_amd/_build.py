"""In-tree builder for the native gfx950 library (``_dllm_native.so``).

Compiles every ``csrc/*.hip`` / ``csrc/*.cpp`` with ``hipcc --offload-arch=gfx950`` into objects under
``build/`` and links one shared object next to this file.  No hipify, no torch JIT cache: the built
``.so`` lives in the source tree so it travels with the repository snapshot to the GPU box.

The library deliberately has no torch headers: it exposes a plain C ABI (raw device pointers + a
``hipStream_t``) that ``_native.py`` calls through ctypes.  It links ``libamdhip64.so.7`` by SONAME; because
Python always imports torch first, the dynamic loader binds it to the HIP runtime torch already loaded,
so kernels, streams and events are shared with PyTorch-ROCm ("Library coexistence").
The RCCL communicator (``csrc/comm.cpp``) is linked against torch's bundled ``librccl.so`` for the same
reason.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD = os.path.join(PKG_DIR, "build")
LIB_NAME = "_dllm_native.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
ARCH = os.environ.get("DLLM_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found; the native library needs ROCm's hipcc")
    return p


def _torch_lib_dir() -> str | None:
    try:
        import torch  # noqa: F401

        d = os.path.join(os.path.dirname(torch.__file__), "lib")
        return d if os.path.isdir(d) else None
    except Exception:  # pragma: no cover
        return None


def sources() -> list[str]:
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".cpp")):
            out.append(os.path.join(CSRC, f))
    return out


def _headers_mtime() -> float:
    m = 0.0
    for f in os.listdir(CSRC):
        if f.endswith((".h", ".hpp")):
            m = max(m, os.path.getmtime(os.path.join(CSRC, f)))
    return m


COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++20", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _compile(src: str, verbose: bool, build_dir: str = BUILD, extra: tuple = ()) -> str:
    obj = os.path.join(build_dir, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime()):
        return obj
    cmd = [_hipcc(), *COMMON_FLAGS, *extra, "-I", CSRC, f"-I{ROCM}/include", "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd.insert(1, "-x")
        cmd.insert(2, "hip")
    if verbose:
        print("[dllm build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


TOOLS = os.path.join(CSRC, "tools")
BIN = os.path.join(PKG_DIR, "bin")


def build_tools(verbose: bool = False, force: bool = False) -> list[str]:
    """Standalone native executables (``csrc/tools/*.cpp`` -> ``bin/dllm_<name>``): separate processes
    without torch, so they link ROCm's own HIP runtime and RCCL."""
    if not os.path.isdir(TOOLS):
        return []
    os.makedirs(BIN, exist_ok=True)
    out = []
    for f in sorted(os.listdir(TOOLS)):
        if not f.endswith(".cpp"):
            continue
        src = os.path.join(TOOLS, f)
        exe = os.path.join(BIN, "dllm_" + f[:-4])
        out.append(exe)
        if not force and os.path.exists(exe) and os.path.getmtime(exe) >= os.path.getmtime(src):
            continue
        cmd = [_hipcc(), "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-x", "hip", src, "-o", exe,
               f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]
        if verbose:
            print("[dllm build]", " ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return out


def build(verbose: bool = False, force: bool = False, jobs: int = 0, variant: str = "", defines: tuple = ()) -> str:
    """Compile all native sources for gfx950 and link ``_dllm_native.so``; returns the library path.

    ``variant`` + ``defines`` (A/B experiments only): build into ``build_<variant>/`` with extra ``-D`` flags and
    link ``_dllm_native_<variant>.so`` next to the production library; load it with ``DLLM_NATIVE_LIB``."""
    build_dir = BUILD + (f"_{variant}" if variant else "")
    lib_path = LIB_PATH.replace(".so", f"_{variant}.so") if variant else LIB_PATH
    extra = tuple(f"-D{d}" for d in defines)
    os.makedirs(build_dir, exist_ok=True)
    if force:
        for f in os.listdir(build_dir):
            os.remove(os.path.join(build_dir, f))
    if not variant:
        build_tools(verbose, force)
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 4, len(srcs))  # the GEMM library is split per layout for this
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose, build_dir, extra), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not force and os.path.exists(lib_path) and os.path.getmtime(lib_path) >= newest:
        return lib_path
    tdir = _torch_lib_dir()
    # -Bsymbolic: the library's own calls bind inside it, so an A/B build loaded next to the production library
    # (scripts/bench_gemm.py --libs) runs its own kernels, not the first-loaded library's same-named entry points
    link = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,-Bsymbolic", *objs, "-o", lib_path + ".tmp"]
    if tdir and os.path.exists(os.path.join(tdir, "librccl.so")):
        # bind RCCL to torch's bundled copy (same SONAME librccl.so.1 as /opt/rocm's)
        link += [f"-L{tdir}", "-l:librccl.so", f"-Wl,-rpath,{tdir}"]
    else:
        link += [f"-L{ROCM}/lib", "-lrccl"]
    if verbose:
        print("[dllm build]", " ".join(link), flush=True)
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(lib_path + ".tmp", lib_path)
    return lib_path


if __name__ == "__main__":
    # python -m dllm._build [-v] [-f] [--variant NAME -DMACRO=VAL ...]
    var = sys.argv[sys.argv.index("--variant") + 1] if "--variant" in sys.argv else ""
    defs = tuple(a[2:] for a in sys.argv if a.startswith("-D"))
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv, variant=var, defines=defs))
