"""Piece hashing of the upload, on the engine.

Mirrors:

  PieceHashAlgorithm / GetPieceHashAlgo   private/piecestore/hash.go:12-26
                                          (BLAKE3 unless overridden by WithPieceHashAlgo)
  pb.NewHashFromAlgorithm(algo) fed by    private/piecestore/upload.go:133,155
  io.TeeReader, Hash: client.hash.Sum(nil) private/piecestore/upload.go:270

The reference hashes each piece while it streams to the storage node, one
byte slice at a time.  Here the hash of every piece of a segment is computed
by the GPU next to the encode, from the copies the encoder already has in
HBM (ec_hash_segments / ec_encode_segments_host_hashed), and the uploader
sends the precomputed 32 bytes.  BLAKE3 is the only algorithm the engine
computes: SHA-256 (the legacy option) is sequential within a piece and is
left to the caller, so asking for it raises.
"""
from __future__ import annotations

import ctypes
import enum

import numpy as np

from . import _native as N
from .eestream import _raise


class PieceHashAlgorithm(enum.IntEnum):
    """pb.PieceHashAlgorithm (storj.io/common/pb)."""
    SHA256 = 0
    BLAKE3 = 1


DEFAULT_ALGORITHM = PieceHashAlgorithm.BLAKE3  # hash.go:25


def _check(algo):
    if PieceHashAlgorithm(algo) != PieceHashAlgorithm.BLAKE3:
        raise NotImplementedError("the engine computes BLAKE3 piece hashes only (SHA256 is the caller's)")


def blake3_host(pieces, algo=DEFAULT_ALGORITHM) -> np.ndarray:
    """[npieces][32] hashes of the rows of a host array [npieces][len]
    (or one 1-D buffer), computed on the GPU (ec_blake3_host)."""
    _check(algo)
    a = np.ascontiguousarray(pieces, dtype=np.uint8)
    if a.ndim == 1:
        a = a.reshape(1, -1)
    npieces, ln = a.shape
    out = np.empty((npieces, 32), dtype=np.uint8)
    rc = N.load().ec_blake3_host(a.ctypes.data if a.size else None, npieces, ln, ln, out.ctypes.data)
    _raise(None, rc)
    return out


def blake3_device(base, npieces: int, piece_len: int, piece_stride: int, hashes, run: int = 0,
                  run_stride: int = 0, stream=None, algo=DEFAULT_ALGORITHM):
    """ec_blake3_pieces on device buffers (torch CUDA tensors or addresses):
    byte t of piece j at base + j*piece_stride + (t//run)*run_stride + t%run
    (run = 0: contiguous).  hashes: npieces*32 device bytes."""
    _check(algo)
    from .eestream import SegmentCodec
    rc = N.load().ec_blake3_pieces(SegmentCodec._addr(base), npieces, piece_stride, piece_len, run, run_stride,
                                   SegmentCodec._addr(hashes), SegmentCodec._stream(stream))
    _raise(None, rc)


def hash_segments(scheme, segs, parity, nseg: int, nstripes: int, hashes, stream=None, algo=DEFAULT_ALGORITHM):
    """ec_hash_segments: BLAKE3 of all n pieces of nseg device-resident
    segments; data pieces are read in place from the stripe-major segments,
    parity pieces from the EC_FLAG_PARITY_ONLY output.  hashes [nseg][n][32]."""
    _check(algo)
    from .eestream import SegmentCodec
    rc = N.load().ec_hash_segments(scheme.ctx, SegmentCodec._addr(segs),
                                   SegmentCodec._addr(parity) if parity is not None else None, nseg, nstripes,
                                   SegmentCodec._addr(hashes), SegmentCodec._stream(stream))
    _raise(scheme.ctx, rc)
