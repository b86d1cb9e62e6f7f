"""Loader for the native libraries built in-tree by :mod:`gnnqc.build`.

* ``libgnnqc_host.so``  - C ABI host runtime (rolling statistics, CRC32C), via ctypes.
* ``libgnnqc_hip.so``   - gfx950 HIP kernels registered as ``torch.ops.gnnqc.*``.

Both live in ``gnnqc/_lib`` so the driver's snapshot carries them to the GPU box.
The HIP library is REQUIRED whenever a tensor is on a GPU: :func:`hip_ops` raises
instead of silently falling back to eager PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "_lib")
HOST_LIB = os.path.join(LIB_DIR, "libgnnqc_host.so")
# GNNQC_HIP_LIB: an alternative build of the HIP library (A/B measurements of compile-time variants,
# scripts/build_chain_variants.py); unset in every normal run
HIP_LIB = os.environ.get("GNNQC_HIP_LIB") or os.path.join(LIB_DIR, "libgnnqc_hip.so")
if not os.path.isabs(HIP_LIB) and not os.path.exists(HIP_LIB):
    # (a relative variant path is taken from the repository root, whatever the working directory)
    HIP_LIB = os.path.join(os.path.dirname(os.path.dirname(LIB_DIR)), HIP_LIB)

_lock = threading.Lock()
_host = None
_hip_loaded = None


def host_lib():
    """ctypes handle of the host library, or None if it has not been built."""
    global _host
    if _host is not None:
        return _host or None
    with _lock:
        if _host is None:
            if os.path.exists(HOST_LIB):
                lib = ctypes.CDLL(HOST_LIB)
                f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
                lib.gq_rolling_stats.argtypes = [f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                 ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_int32]
                lib.gq_rolling_stats.restype = None
                lib.gq_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32]
                lib.gq_crc32c.restype = ctypes.c_uint32
                lib.gq_masked_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
                lib.gq_masked_crc32c.restype = ctypes.c_uint32
                _host = lib
            else:
                _host = False
    return _host or None


def hip_available() -> bool:
    """True if libgnnqc_hip.so is loaded into torch (loads it on first call)."""
    global _hip_loaded
    if _hip_loaded is not None:
        return _hip_loaded
    with _lock:
        if _hip_loaded is None:
            import torch
            if os.path.exists(HIP_LIB):
                torch.ops.load_library(HIP_LIB)
                _hip_loaded = True
                if os.environ.get("GNNQC_DETERMINISTIC", "0") == "1":
                    torch.ops.gnnqc.set_deterministic(True)
            else:
                _hip_loaded = False
    return _hip_loaded


def hip_ops():
    """``torch.ops.gnnqc`` namespace; raises if the HIP extension is missing."""
    import torch
    if not hip_available():
        raise RuntimeError(
            f"gnnqc HIP extension not found at {HIP_LIB}. Build it with "
            "`python -m gnnqc.build` (hipcc --offload-arch=gfx950) before running on a GPU.")
    return torch.ops.gnnqc


# --------------------------------------------------------------- CRC32C
_CRC_TABLE = None


def _crc_table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly = 0x82F63B78
        tab = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            tab.append(c)
        _CRC_TABLE = tab
    return _CRC_TABLE


def crc32c(data: bytes, init: int = 0) -> int:
    lib = host_lib()
    if lib is not None:
        return int(lib.gq_crc32c(data, len(data), init))
    tab = _crc_table()
    c = (~init) & 0xFFFFFFFF
    for b in data:
        c = (c >> 8) ^ tab[(c ^ b) & 0xFF]
    return (~c) & 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


__all__ = ["host_lib", "hip_available", "hip_ops", "crc32c", "masked_crc32c", "LIB_DIR"]
