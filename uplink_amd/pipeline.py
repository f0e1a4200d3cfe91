"""The whole segment transform of upload and download kept in HBM (SURVEY.md
§8f rows 1 and 4 together).

Upload, per segment, as the reference chains it:

  plaintext -> TransformWriterPadded(NewEncrypter(EncAESGCM, key, nonce, 7424))   splitter/splitter.go:156,170
            -> PadReader(stripe size)                                             segmentupload/single.go:236
            -> EncodeSingle for every (piece, stripe)                             segmentupload/encode.go:39-75
            -> BLAKE3 of each piece (TeeReader into the piece hash)              piecestore/upload.go:155,270

Download: Rebuild from k pieces (stripe.go:382-428) -> Transform(NewDecrypter)
-> Unpad to the plain size (streams/store.go:347-382).

Here each arrow is one engine call over a batch of segments on one stream:
ec_pad_segments, ec_gcm_seal_segments_strided (sealing straight into the RS
encoder's padded input), ec_encode_segments, ec_blake3_pieces; and
ec_rebuild_segments_batched, ec_gcm_open_segments_strided.  An encrypted
block (7424 B) is exactly one RS(29,80) stripe, so no data moves between the
stages.
"""
from __future__ import annotations

import numpy as np

from . import _native as N
from .eestream import SegmentCodec, _raise
from .encryption import DEFAULT_BLOCK_SIZE, TAG_SIZE, prepare_keys


def _pad_len(n: int, block: int) -> int:
    return n + 4 + (block - (n + 4) % block) % block


class SegmentGeometry:
    """Sizes of one segment of `plain_len` plaintext bytes through the chain."""

    def __init__(self, plain_len: int, scheme, block_size: int = DEFAULT_BLOCK_SIZE):
        self.plain_len = plain_len
        self.in_block = block_size - TAG_SIZE
        self.block_size = block_size
        self.nblocks = _pad_len(plain_len, self.in_block) // self.in_block       # TransformWriterPadded
        self.enc_len = self.nblocks * block_size                                  # encrypted segment
        self.stripe = scheme.stripe_size()
        self.nstripes = _pad_len(self.enc_len, self.stripe) // self.stripe      # PadReader to the stripe
        self.padded_len = self.nstripes * self.stripe
        self.piece_len = self.nstripes * scheme.erasure_share_size()
        self.plain_cap = self.nblocks * self.in_block                            # plaintext buffer per segment


class DevicePipeline:
    """Batch upload / download transform on device buffers (torch CUDA
    tensors).  `scheme` is an eestream.RSScheme."""

    def __init__(self, scheme, plain_len: int, block_size: int = DEFAULT_BLOCK_SIZE):
        self.scheme = scheme
        self.codec = SegmentCodec(scheme)
        self.g = SegmentGeometry(plain_len, scheme, block_size)
        self._lib = N.load()

    def buffers(self, nseg: int):
        """Allocate the device buffers of a batch: plain [nseg][plain_cap],
        padded encrypted segments [nseg][padded_len], pieces [nseg][n][piece_len],
        hashes [nseg][n][32]."""
        import torch
        g, n = self.g, self.scheme.total_count()
        dev = dict(device="cuda", dtype=torch.uint8)
        return (torch.empty((nseg, g.plain_cap), **dev), torch.empty((nseg, g.padded_len), **dev),
                torch.empty((nseg, n, g.piece_len), **dev), torch.empty((nseg, n, 32), **dev))

    @staticmethod
    def nonces_tensor(nonces):
        import torch
        return torch.from_numpy(np.frombuffer(b"".join(bytes(x)[:12] for x in nonces), dtype=np.uint8).copy()).cuda()

    def upload(self, plain, nseg: int, dev_keys, dev_nonces, enc, pieces, hashes, stream=None):
        """plain [nseg][plain_cap] holds plain_len bytes per segment (the rest
        is overwritten with padding).  Fills enc, pieces and hashes."""
        g, L, s = self.g, self._lib, SegmentCodec._stream(stream)
        a = SegmentCodec._addr
        _raise(None, L.ec_pad_segments(a(plain), nseg, g.plain_cap, g.plain_len, g.in_block, s))
        _raise(None, L.ec_gcm_seal_segments_strided(a(plain), g.plain_cap, nseg, g.nblocks, g.in_block, a(dev_keys),
                                                    a(dev_nonces), a(enc), g.padded_len, s))
        _raise(None, L.ec_pad_segments(a(enc), nseg, g.padded_len, g.enc_len, g.stripe, s))
        self.codec.encode_segments(enc, nseg, g.nstripes, pieces, stream=stream)
        n = self.scheme.total_count()
        _raise(None, L.ec_blake3_pieces(a(pieces), nseg * n, g.piece_len, g.piece_len, 0, 0, a(hashes), s))

    def download(self, nums, pieces, nseg: int, dev_keys, dev_nonces, enc, plain_out, dev_status, stream=None):
        """Rebuild each segment from the pieces numbered `nums` (same set for
        the batch; pieces [nseg][n][piece_len] indexed by number), decrypt
        into plain_out [nseg][plain_cap]; dev_status[g] = -1 or the first
        block of segment g that failed authentication.  The plaintext of a
        segment is plain_out[g, :plain_len]."""
        g, L, s = self.g, self._lib, SegmentCodec._stream(stream)
        a = SegmentCodec._addr
        n = pieces.shape[1]
        base = a(pieces)
        self.codec.rebuild_segments(list(nums), [base + i * g.piece_len for i in nums], g.nstripes, enc, nseg=nseg,
                                    piece_seg_stride=n * g.piece_len, out_seg_stride=g.padded_len, stream=stream)
        _raise(None, L.ec_gcm_open_segments_strided(a(enc), g.padded_len, nseg, g.nblocks, g.in_block, a(dev_keys),
                                                    a(dev_nonces), a(plain_out), g.plain_cap, a(dev_status), s))

    @staticmethod
    def prepare_keys(keys, stream=None):
        return prepare_keys(keys, stream=stream)
