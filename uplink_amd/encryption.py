"""Segment encryption on the engine: the AES-256-GCM
transform of storj.io/common/encryption as the stream layer uses it.

Mirrors:

  increment / nonce_for_position   encryption.Increment; splitter/common.go:27-32,
                                   streams/store.go:264-270 (deriveContentNonce)
  AESGCMEncrypter                  encryption.NewEncrypter(EncAESGCM, key, nonce, BlockSize)
                                   splitter/splitter.go:156; InBlockSize = BlockSize-16
  encrypt_segment                  encryption.TransformWriterPadded(buf, enc)  splitter.go:170
  AESGCMDecrypter/decrypt_segment  decryptRanger: NewDecrypter, Transform, Unpad
                                   streams/store.go:347-382

Every block is sealed or opened by the GPU (ec_gcm_*); a block whose tag
does not verify raises DecryptionFailed ("cipher: message authentication
failed", Go's crypto/cipher error) naming the block.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from .eestream import _raise, pad, unpad

TAG_SIZE = 16
DEFAULT_BLOCK_SIZE = 29 * 256  # project.go:84


class DecryptionFailed(Exception):
    def __init__(self, block: int):
        super().__init__(f"cipher: message authentication failed (block {block})")
        self.block = block


def increment(nonce: bytes, amount: int) -> bytes:
    """encryption.Increment: little-endian add with carry (wraps silently)."""
    if amount < 0:
        raise ValueError("amount was negative")
    b = bytearray(nonce)
    for i in range(len(b)):
        if not amount:
            break
        s = b[i] + (amount & 0xFF)
        b[i] = s & 0xFF
        amount = (amount >> 8) + (s >> 8)
    return bytes(b)


def nonce_for_position(part_number: int, index: int) -> bytes:
    """24-byte storj.Nonce for a segment position (splitter/common.go:27-32)."""
    return increment(bytes(24), (part_number << 32) | (index + 1))


def _key(key) -> bytes:
    key = bytes(key)
    if len(key) != 32:
        raise ValueError("AES-256-GCM needs a 32-byte key")
    return key


class AESGCMEncrypter:
    """NewEncrypter(EncAESGCM, key, nonce, encrypted_block_size)."""

    def __init__(self, key, starting_nonce, encrypted_block_size: int = DEFAULT_BLOCK_SIZE):
        if encrypted_block_size <= TAG_SIZE:
            raise ValueError(f"encrypted block size {encrypted_block_size} too small")
        self.key = _key(key)
        self.nonce = bytes(starting_nonce)[:12]  # AESGCMNonce = first 12 bytes of storj.Nonce
        self.block_size = encrypted_block_size

    def in_block_size(self) -> int:
        return self.block_size - TAG_SIZE

    def out_block_size(self) -> int:
        return self.block_size

    def transform(self, padded) -> bytes:
        """Seal every InBlockSize block of `padded` (block b under nonce + b)."""
        a = np.ascontiguousarray(np.frombuffer(bytes(padded), dtype=np.uint8))
        ib = self.in_block_size()
        if a.size % ib:
            raise ValueError(f"input is not a multiple of the block size {ib}")
        nb = a.size // ib
        out = np.empty(nb * self.block_size, dtype=np.uint8)
        rc = N.load().ec_gcm_seal_host(self.key, self.nonce, a.ctypes.data if a.size else None, nb, ib,
                                       out.ctypes.data if out.size else None)
        _raise(None, rc)
        return out.tobytes()


class AESGCMDecrypter(AESGCMEncrypter):
    """NewDecrypter(EncAESGCM, key, nonce, encrypted_block_size)."""

    def in_block_size(self) -> int:
        return self.block_size

    def out_block_size(self) -> int:
        return self.block_size - TAG_SIZE

    def transform(self, cipher) -> bytes:
        a = np.ascontiguousarray(np.frombuffer(bytes(cipher), dtype=np.uint8))
        if a.size % self.block_size:
            raise ValueError(f"input is not a multiple of the block size {self.block_size}")
        nb = a.size // self.block_size
        ib = self.block_size - TAG_SIZE
        out = np.empty(nb * ib, dtype=np.uint8)
        bad = ctypes.c_longlong(-1)
        rc = N.load().ec_gcm_open_host(self.key, self.nonce, a.ctypes.data if a.size else None, nb, ib,
                                       out.ctypes.data if out.size else None, ctypes.byref(bad))
        if rc == N.EC_ERR_AUTH:
            raise DecryptionFailed(bad.value)
        _raise(None, rc)
        return out.tobytes()


def encrypt_segment(plain, key, nonce, block_size: int = DEFAULT_BLOCK_SIZE) -> bytes:
    """TransformWriterPadded(buf, NewEncrypter(...)): PadReader padding to
    InBlockSize, then one GCM seal per block."""
    enc = AESGCMEncrypter(key, nonce, block_size)
    return enc.transform(pad(bytes(plain), enc.in_block_size()))


def decrypt_segment(cipher, key, nonce, plain_size: int | None = None, block_size: int = DEFAULT_BLOCK_SIZE) -> bytes:
    """decryptRanger's Transform + Unpad: plain_size when known (store.go:381),
    else the padding trailer."""
    padded = AESGCMDecrypter(key, nonce, block_size).transform(cipher)
    return padded[:plain_size] if plain_size is not None else unpad(padded)


def prepare_keys(keys, dev_buf=None, stream=None):
    """ec_gcm_prepare_keys into a device buffer (torch uint8 tensor allocated
    when dev_buf is None); returns it."""
    import torch
    from .eestream import SegmentCodec
    keys = [_key(k) for k in keys]
    nbytes = len(keys) * N.load().ec_gcm_key_bytes()
    if dev_buf is None:
        dev_buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda")
    host = np.frombuffer(b"".join(keys), dtype=np.uint8)
    rc = N.load().ec_gcm_prepare_keys(host.ctypes.data, len(keys), SegmentCodec._addr(dev_buf),
                                      SegmentCodec._stream(stream))
    _raise(None, rc)
    return dev_buf


def seal_segments(plain, nseg: int, nblocks: int, in_block: int, dev_keys, dev_nonces, out, stream=None):
    """ec_gcm_seal_segments on device buffers: [nseg][nblocks*in_block] ->
    [nseg][nblocks*(in_block+16)]."""
    from .eestream import SegmentCodec as C
    rc = N.load().ec_gcm_seal_segments(C._addr(plain), nseg, nblocks, in_block, C._addr(dev_keys),
                                       C._addr(dev_nonces), C._addr(out), C._stream(stream))
    _raise(None, rc)


def open_segments(cipher, nseg: int, nblocks: int, in_block: int, dev_keys, dev_nonces, out, dev_status,
                  stream=None):
    """ec_gcm_open_segments; dev_status[g] = -1 or the first failing block."""
    from .eestream import SegmentCodec as C
    rc = N.load().ec_gcm_open_segments(C._addr(cipher), nseg, nblocks, in_block, C._addr(dev_keys),
                                       C._addr(dev_nonces), C._addr(out), C._addr(dev_status), C._stream(stream))
    _raise(None, rc)
