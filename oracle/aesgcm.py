"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by uplink_amd/).

ctypes binding of oracle/aesgcm_oracle.c: storj/uplink's segment encryption
(AES-256-GCM blocks of BlockSize - 16 plaintext bytes, per-block nonces,
PadReader padding), restated from storj.io/common/encryption (go.mod:14) on
top of OpenSSL's AES-256-GCM.  Pinned by the GCM specification's test cases
(tests/golden/aesgcm_vectors.json).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import oracle as _o

LIB_PATH = os.path.join(_o.HERE, "build", "libaesgcm_oracle.so")
_lib = None
TAG = 16


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            _o.build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.ag_increment.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint64]
        L.ag_seal.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp]
        L.ag_open.argtypes = [vp, vp, vp, ctypes.c_size_t, vp]
        for f in (L.ag_encrypt_blocks, L.ag_decrypt_blocks):
            f.argtypes = [vp, vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, ctypes.c_int]
            f.restype = ctypes.c_int64
        _lib = L
    return _lib


def _buf(b) -> np.ndarray:
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b)
    return a if a.size else np.zeros(1, dtype=np.uint8)


def increment(nonce: bytes, amount: int) -> bytes:
    """encryption.Increment / incrementBytes: little-endian add with carry."""
    a = bytearray(nonce)
    buf = (ctypes.c_uint8 * len(a)).from_buffer(a)
    lib().ag_increment(ctypes.addressof(buf), len(a), amount)
    return bytes(a)


def nonce_for_position(part: int, index: int) -> bytes:
    """splitter/common.go:27-32 (== streams/store.go:264-270): 24-byte nonce."""
    return increment(bytes(24), (part << 32) | (index + 1))


def seal(key: bytes, nonce12: bytes, plain: bytes, aad: bytes = b"") -> bytes:
    out = np.empty(len(plain) + TAG, dtype=np.uint8)
    p, a = _buf(plain), _buf(aad)
    rc = lib().ag_seal(key, nonce12, a.ctypes.data, len(aad), p.ctypes.data, len(plain), out.ctypes.data)
    assert rc == 0
    return out.tobytes()


def open_(key: bytes, nonce12: bytes, sealed: bytes) -> bytes | None:
    n = len(sealed) - TAG
    out = np.empty(max(n, 1), dtype=np.uint8)
    s = _buf(sealed)
    rc = lib().ag_open(key, nonce12, s.ctypes.data, n, out.ctypes.data)
    return out[:n].tobytes() if rc == 0 else None


def encrypt_blocks(key: bytes, nonce: bytes, padded: np.ndarray, in_block: int, threads: int = 1,
                   out: np.ndarray | None = None) -> np.ndarray:
    """Encrypter.Transform over the padded plaintext: [nblocks][in_block+16]
    (into `out` when given, e.g. a pre-faulted buffer for timing)."""
    padded = np.ascontiguousarray(padded, dtype=np.uint8).reshape(-1)
    nb = padded.size // in_block
    assert nb * in_block == padded.size
    if out is None:
        out = np.empty((nb, in_block + TAG), dtype=np.uint8)
    rc = lib().ag_encrypt_blocks(key, nonce[:12], padded.ctypes.data, nb, in_block, out.ctypes.data, threads)
    assert rc == -1, rc
    return out


def decrypt_blocks(key: bytes, nonce: bytes, cipher: np.ndarray, in_block: int, threads: int = 1):
    """Decrypter.Transform: (plaintext [nblocks*in_block], first failing block or -1)."""
    cipher = np.ascontiguousarray(cipher, dtype=np.uint8).reshape(-1)
    nb = cipher.size // (in_block + TAG)
    out = np.empty(max(nb * in_block, 1), dtype=np.uint8)
    bad = lib().ag_decrypt_blocks(key, nonce[:12], cipher.ctypes.data, nb, in_block, out.ctypes.data, threads)
    return out[:nb * in_block], int(bad)


def encrypt_segment(plain: bytes, key: bytes, nonce24: bytes, block_size: int = 29 * 256, threads: int = 1):
    """TransformWriterPadded(NewEncrypter(EncAESGCM, key, nonce, block_size)):
    pad to InBlockSize = block_size - 16 with the PadReader rule, then seal
    every block.  Returns the encrypted segment bytes (nblocks*block_size)."""
    in_block = block_size - TAG
    padded = _o.pad(np.frombuffer(bytes(plain), dtype=np.uint8), in_block)
    return encrypt_blocks(key, nonce24, padded, in_block, threads).reshape(-1)


def decrypt_segment(cipher, key: bytes, nonce24: bytes, plain_size: int, block_size: int = 29 * 256,
                    threads: int = 1):
    """Transform(NewDecrypter(...)) + Unpad(plain_size) (store.go:377-381);
    None when a block fails authentication."""
    in_block = block_size - TAG
    out, bad = decrypt_blocks(key, nonce24, np.frombuffer(bytes(cipher), dtype=np.uint8), in_block, threads)
    return None if bad >= 0 else out[:plain_size].tobytes()
