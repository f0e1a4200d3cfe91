"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by uplink_amd/).

ctypes binding of oracle/blake3_oracle.c, the CPU restatement of BLAKE3-256
(github.com/zeebo/blake3 v0.2.3, go.mod:29), the piece hash of
private/piecestore/upload.go:133,155,270.  Pinned by the official test
vectors in tests/golden/blake3_vectors.json.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import oracle as _o

LIB_PATH = os.path.join(_o.HERE, "build", "libblake3_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            _o.build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.b3_hash.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.b3_hash_many.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, u8p, ctypes.c_int]
        _lib = L
    return _lib


def _arr(data) -> np.ndarray:
    a = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1)
    return a if a.size else np.zeros(1, dtype=np.uint8)[:0]


def blake3(data) -> bytes:
    """BLAKE3-256 of `data` (32 bytes), what zeebo/blake3's Sum(nil) returns."""
    a = _arr(data)
    buf = a if a.size else np.zeros(1, dtype=np.uint8)
    out = np.empty(32, dtype=np.uint8)
    lib().b3_hash(_o._p(buf), a.size, _o._p(out))
    return out.tobytes()


def blake3_many(pieces: np.ndarray, threads: int = 1) -> np.ndarray:
    """[npieces][32] hashes of the rows of a C-contiguous [npieces][len] array."""
    pieces = np.ascontiguousarray(pieces, dtype=np.uint8)
    npieces, ln = pieces.shape
    out = np.empty((npieces, 32), dtype=np.uint8)
    src = pieces if pieces.size else np.zeros((max(npieces, 1), 1), dtype=np.uint8)
    lib().b3_hash_many(_o._p(src), npieces, src.shape[1] if ln else 0, ln, _o._p(out), threads)
    return out
