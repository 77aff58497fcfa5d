"""ctypes binding of ``_dllm_native.so`` (the gfx950 kernels + RCCL communicator).

Import order matters: ``torch`` is imported first so the library's ``libamdhip64.so.7`` / ``librccl.so.1``
dependencies resolve to the copies PyTorch-ROCm already loaded (one HIP runtime per process).

Policy (no silent fallbacks on a GPU): ``lib()`` raises if the library cannot be loaded and a GPU is
present.  CPU tensors never reach this module — the op layer routes them to the torch reference path.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load)

from . import _build

_LOCK = threading.Lock()
_LIB: ctypes.CDLL | None = None
_ERR: str | None = None

c_int, c_long, c_float, c_void_p, c_ull = ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_void_p, ctypes.c_ulonglong

# bumped with every signature or stream-semantics change below (csrc/elementwise.hip dllm_abi_version): a stale library fails loudly
ABI_VERSION = 13

_SIGS = {
    "dllm_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_long,
                          c_void_p, c_void_p, c_long, c_int, c_int, c_int, c_float, c_float, c_int, c_int, c_void_p,
                          c_float, c_float, c_float, c_float, c_float, c_int, c_void_p, c_void_p, c_int, c_void_p,
                          c_void_p, c_int, c_int, c_int]),
    "dllm_gemm_path": (c_int, [c_int, c_int, c_int, c_int, c_int, c_long, c_long, c_long]),
    "dllm_queue_shared": (c_int, [c_void_p, c_void_p, c_int]),
    "dllm_queue_reserve": (c_int, [c_void_p, c_int, c_int]),
    "dllm_gemm_pair": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_float, c_float,
                               c_float, c_float, c_float, c_int, c_void_p]),
    "dllm_rng_normal": (c_int, [c_void_p, c_int, c_long, c_ull, c_ull, c_float, c_void_p]),
    "dllm_rng_normal_devseed": (c_int, [c_void_p, c_int, c_long, c_void_p, c_ull, c_float, c_void_p]),
    "dllm_rng_normal_bf16_pair": (c_int, [c_void_p, c_void_p, c_long, c_ull, c_void_p, c_ull, c_ull, c_float, c_float,
                                          c_void_p]),
    "dllm_rng_normal_bf16_t": (c_int, [c_void_p, c_void_p, c_long, c_long, c_ull, c_void_p, c_ull, c_float, c_void_p]),
    "dllm_sgd_step": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_long, c_float, c_float, c_void_p]),
    "dllm_sgd_step_stream": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_long, c_float, c_float, c_int,
                                     c_void_p]),
    "dllm_adam_step": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_long, c_float, c_float,
                               c_float, c_float, c_float, c_int, c_float, c_void_p]),
    "dllm_sgd_split_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_long, c_float, c_float, c_void_p]),
    "dllm_split_master": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p]),
    "dllm_adam_split_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_long, c_float,
                                     c_float, c_float, c_float, c_float, c_int, c_float, c_void_p]),
    "dllm_cast": (c_int, [c_void_p, c_int, c_void_p, c_int, c_long, c_void_p]),
    "dllm_split3": (c_int, [c_void_p, c_long, c_long, c_long, c_void_p, c_int, c_int, c_void_p]),
    "dllm_transpose_bf16": (c_int, [c_void_p, c_long, c_void_p, c_long, c_long, c_long, c_void_p]),
    "dllm_occupy": (c_int, [c_int, c_int, c_float, c_void_p, c_void_p]),
    "dllm_abi_version": (c_int, []),
}
_OPTIONAL_SIGS: dict = {}


def register_optional(name: str, restype, argtypes) -> None:
    """Declare a symbol that newer library builds export (bound lazily if present)."""
    _OPTIONAL_SIGS[name] = (restype, argtypes)
    if _LIB is not None and hasattr(_LIB, name):
        f = getattr(_LIB, name)
        f.restype, f.argtypes = restype, argtypes


def _load() -> ctypes.CDLL:
    path = os.environ.get("DLLM_NATIVE_LIB") or _build.LIB_PATH  # alternate build (A/B experiments)
    if path == _build.LIB_PATH and (not os.path.exists(path) or os.environ.get("DLLM_REBUILD") == "1"):
        _build.build()
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in {**_SIGS, **_OPTIONAL_SIGS}.items():
        if not hasattr(lib, name):
            if name in _SIGS:
                raise RuntimeError(f"{path} lacks symbol {name}; rebuild with python -m dllm._build -f")
            continue
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    if lib.dllm_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{path} has C ABI {lib.dllm_abi_version()}, expected {ABI_VERSION}; "
                           "rebuild with python -m dllm._build -f")
    return lib


def lib() -> ctypes.CDLL:
    global _LIB, _ERR
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            try:
                _LIB = _load()
            except Exception as e:  # pragma: no cover - exercised on broken installs
                _ERR = f"{type(e).__name__}: {e}"
                raise RuntimeError(f"dllm native library unavailable: {_ERR}") from e
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except RuntimeError:
        return False


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


DT = {torch.bfloat16: 0, torch.float32: 1}


def dtype_code(t: torch.dtype) -> int:
    if t not in DT:
        raise TypeError(f"unsupported dtype {t}; native kernels take bf16 or fp32")
    return DT[t]
