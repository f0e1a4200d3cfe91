"""Host-side mirror of storj/uplink's private/eestream ErasureScheme surface,
backed by the MI355X engine (libuplink_ec.so, include/uplink_ec.h).

Same names, argument meaning and error behaviour as the Go reference, so the
parity tests read like the reference's own tests:

  new_fec / FEC                  eestream.NewFEC               private/eestream/fec.go:15-17
  Share                          infectious.Share              private/eestream/fec.go:9
  RSScheme (ErasureScheme)       rsScheme                      private/eestream/rs.go:11-61
  UnsafeRSScheme                 unsafeRSScheme (no Correct)   private/eestream/unsafe_rs.go:11-73
    .encode / .encode_single / .decode / .rebuild / sizes     scheme.go:13-41
  RedundancyStrategy             encode.go:23-99 (threshold validation + errors)
  calc_piece_size                CalcPieceSize                 encode.go:272-281
  EncodedReader                  segmentupload.EncodedReader   segmentupload/encode.go:16-75
  pad / unpad                    encryption.PadReader/Unpad    (storj.io/common)
  RSScheme.encode_stripes / .rebuild_stripes
                                 host-memory batch forms used by streams.py
  SegmentCodec                   batch forms of the per-(piece, stripe) EncodeSingle loop
                                 (segmentupload/single.go:228-238) and of the per-stripe
                                 Rebuild loop (stripe.go:382-428) on device-resident buffers

Every byte of share data is computed on the GPU; there is no CPU fallback
(the library raises if it is missing, ec_create fails without a GPU).
"""
from __future__ import annotations

import ctypes
import io
from dataclasses import dataclass
from typing import Callable, Iterable, List, Optional

import numpy as np

from . import _native as N


# ------------------------------------------------------------------ errors
class EEStreamError(Exception):
    """errs.Class("eestream") (private/eestream/common.go:13): messages are
    prefixed with "eestream: "."""

    def __init__(self, msg: str):
        super().__init__("eestream: " + msg)


class InfectiousError(Exception):
    """An error returned by the erasure code itself (infectious)."""

    code = None


class NotEnoughShares(InfectiousError):
    """infectious.NotEnoughShares (tested by stripe.go:446-449)."""


class TooManyErrors(InfectiousError):
    """infectious.TooManyErrors (tested by stripe.go:446-449)."""


class DeviceError(RuntimeError):
    pass


def _raise(ctx, code: int, arg: int = 0):
    if code == N.EC_OK:
        return
    buf = ctypes.create_string_buffer(256)
    N.load().ec_format_error(ctx, code, arg, buf, len(buf))
    msg = buf.value.decode()
    if code == N.EC_ERR_NOT_ENOUGH_SHARES:
        raise NotEnoughShares(msg)
    if code == N.EC_ERR_TOO_MANY_ERRORS:
        raise TooManyErrors(msg)
    if code == N.EC_ERR_DEVICE:
        raise DeviceError(msg)
    e = InfectiousError(msg)
    e.code = code
    raise e


def _u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf, dtype=np.uint8)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


# ------------------------------------------------------------------ shares
@dataclass
class Share:
    """infectious.Share{Number int; Data []byte}."""

    number: int
    data: np.ndarray

    def deep_copy(self) -> "Share":
        return Share(self.number, np.array(self.data, dtype=np.uint8, copy=True))


# ------------------------------------------------------------------ FEC
class FEC:
    """Parameters of a (k, n) code: eestream.NewFEC / infectious.NewFEC."""

    def __init__(self, k: int, n: int):
        if k <= 0 or n <= 0 or k > 256 or n > 256 or k > n:
            raise InfectiousError("requires 1 <= k <= n <= 256")
        self.k, self.n = k, n

    def required(self) -> int:
        return self.k

    def total(self) -> int:
        return self.n


def new_fec(k: int, n: int) -> FEC:
    return FEC(k, n)


# ------------------------------------------------------------------ scheme
class RSScheme:
    """ErasureScheme backed by the GPU engine (mirrors rsScheme, rs.go:11-61)."""

    def __init__(self, fc: FEC, erasure_share_size: int):
        self._lib = N.load()
        self.fc = fc
        self.ess = erasure_share_size
        self._ctx = ctypes.c_void_p()
        rc = self._lib.ec_create(fc.k, fc.n, erasure_share_size, ctypes.byref(self._ctx))
        _raise(None, rc)

    def close(self):
        if self._ctx:
            self._lib.ec_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    # -- sizes (rs.go:47-61)
    def erasure_share_size(self) -> int:
        return self.ess

    def stripe_size(self) -> int:
        return self.ess * self.fc.k

    def total_count(self) -> int:
        return self.fc.n

    def required_count(self) -> int:
        return self.fc.k

    def generator(self) -> np.ndarray:
        g = np.zeros(self.fc.n * self.fc.k, dtype=np.uint8)
        self._lib.ec_generator(self._ctx, _ptr(g))
        return g.reshape(self.fc.n, self.fc.k)

    # -- EncodeSingle (rs.go:21-23)
    def encode_single(self, inp, out: np.ndarray, num: int) -> None:
        a = _u8(inp)
        if not (isinstance(out, np.ndarray) and out.dtype == np.uint8 and out.flags["C_CONTIGUOUS"]):
            raise TypeError("out must be a contiguous uint8 numpy array")
        rc = self._lib.ec_encode_single(self._ctx, _ptr(a), a.size, _ptr(out), out.size, num)
        _raise(self._ctx, rc, (a.size // self.fc.k) if self.fc.k else 0)

    # -- Encode (rs.go:25-30): out(num, data) for every share, data valid only
    #    during the callback
    def encode(self, inp, out: Callable[[int, np.ndarray], None]) -> None:
        a = _u8(inp)
        k, n = self.fc.k, self.fc.n
        if a.size % k:
            _raise(self._ctx, N.EC_ERR_INPUT_LENGTH)
        bs = a.size // k
        buf = np.zeros(max(n * bs, 1), dtype=np.uint8)
        rc = self._lib.ec_encode(self._ctx, _ptr(a), a.size, _ptr(buf))
        _raise(self._ctx, rc)
        for i in range(n):
            out(i, buf[i * bs:(i + 1) * bs])

    def _share_arrays(self, shares: List[Share]):
        lens = {len(s.data) for s in shares}
        if len(lens) > 1:
            _raise(self._ctx, N.EC_ERR_SHARE_SIZE)
        ln = lens.pop() if lens else 0
        datas = [np.ascontiguousarray(s.data, dtype=np.uint8) for s in shares]
        nums = (ctypes.c_int * max(len(shares), 1))(*[s.number for s in shares])
        ptrs = (ctypes.c_void_p * max(len(shares), 1))(*[d.ctypes.data for d in datas])
        return ln, datas, nums, ptrs

    def _resort(self, shares: List[Share], nums, ptrs, datas):
        # the C side sorted (nums, ptrs) in place like infectious sorts []Share
        by_ptr = {d.ctypes.data: (s, d) for s, d in zip(shares, datas)}
        shares[:] = [Share(nums[i], by_ptr[ptrs[i]][1]) for i in range(len(shares))]

    # -- Rebuild (rs.go:40-45): out(share) for the k data shares, in order
    def rebuild(self, shares: List[Share], out: Optional[Callable[[Share], None]]) -> None:
        ln, datas, nums, ptrs = self._share_arrays(shares)
        k = self.fc.k
        buf = np.zeros(max(k * ln, 1), dtype=np.uint8)
        rc = self._lib.ec_rebuild(self._ctx, len(shares), nums, ptrs, ln, _ptr(buf))
        if len(shares) >= k:
            self._resort(shares, nums, ptrs, datas)
        _raise(self._ctx, rc)
        if out is not None:
            for i in range(k):
                out(Share(i, buf[i * ln:(i + 1) * ln]))

    # -- Decode (rs.go:32-38): Correct + Rebuild, returns k*len bytes; the
    #    shares are sorted and corrected in place
    def decode(self, out: Optional[np.ndarray], shares: List[Share]) -> np.ndarray:
        ln, datas, nums, ptrs = self._share_arrays(shares)
        k = self.fc.k
        need = k * ln
        dst = out if (out is not None and out.size >= need) else np.empty(max(need, 1), dtype=np.uint8)
        dst = dst[:need] if need else dst[:0]
        # written only once the decode has succeeded (the C side copies out last)
        target = dst if dst.flags["C_CONTIGUOUS"] else np.empty(max(need, 1), dtype=np.uint8)
        rc = self._lib.ec_decode(self._ctx, len(shares), nums, ptrs, ln, _ptr(target))
        if len(shares) >= k:
            self._resort(shares, nums, ptrs, datas)
        _raise(self._ctx, rc)
        if target is not dst:
            dst[:] = target[:need]
        return dst


    # -- batch forms used by the stream layer (streams.py): whole runs of
    #    stripes per engine call instead of one call per (piece, stripe)
    def encode_stripes(self, data) -> np.ndarray:
        """EncodeSingle for every piece of len(data)/StripeSize stripes:
        returns [n][stripes*ess] (host memory in and out)."""
        a = _u8(data)
        stripe = self.stripe_size()
        if a.size % stripe:
            _raise(self._ctx, N.EC_ERR_INPUT_LENGTH)
        m = a.size // stripe
        out = np.empty((self.fc.n, m * self.ess), dtype=np.uint8)
        if m:
            _raise(self._ctx, self._lib.ec_encode_segments_host(self._ctx, _ptr(a), 1, m, _ptr(out), 0))
        return out

    def rebuild_stripes(self, nums, pieces, nstripes: int) -> np.ndarray:
        """Rebuild over `nstripes` stripes at once from the shares of pieces
        `nums` (each nstripes*ess host bytes): infectious' share choice, one
        decode matrix for the run; returns the stripes (nstripes*k*ess)."""
        arrs = [np.ascontiguousarray(p, dtype=np.uint8) for p in pieces]
        if len(arrs) != len(nums):
            raise ValueError("nums and pieces differ in length")
        out = np.empty(max(nstripes * self.fc.k * self.ess, 1), dtype=np.uint8)
        c_nums = (ctypes.c_int * max(len(nums), 1))(*nums)
        c_ptrs = (ctypes.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
        if nstripes:
            _raise(self._ctx, self._lib.ec_rebuild_segments_host(self._ctx, len(nums), c_nums, c_ptrs, nstripes, 1, 0,
                                                                 _ptr(out)))
        return out[:nstripes * self.fc.k * self.ess]


def new_rs_scheme(fc: FEC, erasure_share_size: int) -> RSScheme:
    return RSScheme(fc, erasure_share_size)


class UnsafeRSScheme(RSScheme):
    """unsafeRSScheme (unsafe_rs.go:11-73): Decode is Rebuild into out (the k
    data shares at number * ess), without error correction."""

    def decode(self, out: Optional[np.ndarray], shares: List[Share]) -> np.ndarray:
        ln = len(shares[0].data) if shares else 0
        need = self.fc.k * ln
        dst = out[:need] if (out is not None and out.size >= need) else np.zeros(max(need, 1), dtype=np.uint8)[:need]

        def put(sh: Share):
            dst[sh.number * ln:(sh.number + 1) * ln] = sh.data
        self.rebuild(shares, put)
        return dst


def new_unsafe_rs_scheme(fc: FEC, erasure_share_size: int) -> UnsafeRSScheme:
    """NewUnsafeRSScheme (unsafe_rs.go:16-19)."""
    return UnsafeRSScheme(fc, erasure_share_size)


# ------------------------------------------------------------------ strategy
class RedundancyStrategy:
    """ErasureScheme with repair / optimal thresholds (encode.go:23-99)."""

    def __init__(self, es: RSScheme, repair_threshold: int = 0, optimal_threshold: int = 0):
        if repair_threshold == 0:
            repair_threshold = es.total_count()
        if optimal_threshold == 0:
            optimal_threshold = es.total_count()
        if repair_threshold < 0:
            raise EEStreamError("negative repair threshold")
        if 0 < repair_threshold < es.required_count():
            raise EEStreamError("repair threshold less than required count")
        if repair_threshold > es.total_count():
            raise EEStreamError("repair threshold greater than total count")
        if optimal_threshold < 0:
            raise EEStreamError("negative optimal threshold")
        if 0 < optimal_threshold < es.required_count():
            raise EEStreamError("optimal threshold less than required count")
        if optimal_threshold > es.total_count():
            raise EEStreamError("optimal threshold greater than total count")
        if repair_threshold > optimal_threshold:
            raise EEStreamError("repair threshold greater than optimal threshold")
        self.scheme = es
        self._repair = repair_threshold
        self._optimal = optimal_threshold

    def repair_threshold(self) -> int:
        return self._repair

    def optimal_threshold(self) -> int:
        return self._optimal

    def __getattr__(self, name):  # embeds ErasureScheme like the Go struct
        return getattr(self.scheme, name)


def new_redundancy_strategy(es: RSScheme, repair: int, optimal: int) -> RedundancyStrategy:
    return RedundancyStrategy(es, repair, optimal)


def new_redundancy_strategy_from_storj(required: int, repair: int, optimal: int, total: int,
                                       share_size: int) -> RedundancyStrategy:
    """NewRedundancyStrategyFromStorj (encode.go:78-87)."""
    try:
        fc = new_fec(required, total)
    except InfectiousError as e:
        raise EEStreamError(str(e))
    return RedundancyStrategy(RSScheme(fc, share_size), repair, optimal)


def calc_piece_size(data_size: int, scheme) -> int:
    """CalcPieceSize (encode.go:272-281): PadReader's +4 byte length trailer."""
    stripe = scheme.stripe_size()
    stripes = (data_size + 4 + stripe - 1) // stripe
    return stripes * stripe // scheme.required_count()


# ------------------------------------------------------------------ padding
def pad(data: bytes, block_size: int) -> bytes:
    """encryption.PadReader semantics: p = 4 +
    (bs - (len+4) % bs) % bs pad bytes equal to byte(p), the last 4 bytes the
    big-endian uint32 p."""
    p = 4 + (block_size - (len(data) + 4) % block_size) % block_size
    tail = bytearray([p & 0xFF] * p)
    tail[-4:] = p.to_bytes(4, "big")
    return bytes(data) + bytes(tail)


def unpad(padded: bytes) -> bytes:
    """encryption.UnpadSlow: strip the trailer written by pad."""
    if len(padded) < 4:
        raise EEStreamError("invalid padding")
    p = int.from_bytes(padded[-4:], "big")
    if p < 4 or p > len(padded):
        raise EEStreamError("invalid padding")
    return bytes(padded[:-p])


# ------------------------------------------------------------------ readers
class EncodedReader(io.RawIOBase):
    """segmentupload.EncodedReader (segmentupload/encode.go:16-75): the piece
    `num` of a padded segment stream, one EncodeSingle per stripe."""

    def __init__(self, r, rs, num: int):
        super().__init__()
        self._r = r
        self._rs = rs
        self._num = num
        self._stripe = rs.stripe_size()
        self._share = np.zeros(rs.erasure_share_size(), dtype=np.uint8)
        self._avail = 0
        self._err: Optional[Exception] = None
        self._eof = False

    def readable(self):
        return True

    def _read_full(self, n):
        chunks, got = [], 0
        while got < n:
            b = self._r.read(n - got)
            if not b:
                break
            chunks.append(b)
            got += len(b)
        return b"".join(chunks)

    def read(self, size: int = -1) -> bytes:
        if self._err is not None:
            raise self._err
        out = bytearray()
        want = size if size is not None and size >= 0 else 1 << 62
        while len(out) < want:
            if self._avail == 0:
                if self._eof:
                    break
                stripe = self._read_full(self._stripe)
                if len(stripe) == 0:
                    self._eof = True
                    break
                if len(stripe) < self._stripe:
                    self._err = EOFError("unexpected EOF")
                    raise self._err
                try:
                    self._rs.encode_single(np.frombuffer(stripe, dtype=np.uint8), self._share, self._num)
                except Exception as e:
                    self._err = e
                    raise
                self._avail = len(self._share)
            off = len(self._share) - self._avail
            take = min(self._avail, want - len(out))
            out += self._share[off:off + take].tobytes()
            self._avail -= take
        return bytes(out)


def new_encoded_reader(r, rs, num: int) -> EncodedReader:
    return EncodedReader(r, rs, num)


# ------------------------------------------------------------------ device batches
class SegmentCodec:
    """Batch forms on device-resident buffers (torch CUDA tensors or raw
    device pointers): whole segments at once instead of per (piece, stripe).

    encode_segments(segs, nseg, nstripes, pieces, parity_only=False, stream=None)
        segs   [nseg][nstripes][k][ess]  (padded, stripe-major)
        pieces [nseg][n][nstripes*ess]   ([nseg][n-k][...] when parity_only)
    rebuild_segments(nums, piece_ptrs, nstripes, out, nseg=1, piece_seg_stride=0,
                     out_seg_stride=0, stream=None)
        out    [nseg][nstripes][k][ess]
    rebuild_segments_sets(sets, nstripes, outs, stream=None)
    decode_segments_sets(sets, nstripes, outs, stream=None)
        sets   one (nums, piece_ptrs) per segment: each segment with its own share set
        outs   one [nstripes][k][ess] output per segment
    """

    def __init__(self, scheme: RSScheme):
        self.scheme = scheme
        self._lib = scheme._lib

    @staticmethod
    def _addr(x):
        return x.data_ptr() if hasattr(x, "data_ptr") else int(x)

    @staticmethod
    def _stream(stream):
        if stream is None:
            try:
                import torch
                return torch.cuda.current_stream().cuda_stream
            except Exception:
                return None
        return stream.cuda_stream if hasattr(stream, "cuda_stream") else stream

    def encode_segments(self, segs, nseg: int, nstripes: int, pieces, parity_only: bool = False, stream=None):
        flags = N.EC_FLAG_PARITY_ONLY if parity_only else 0
        rc = self._lib.ec_encode_segments(self.scheme.ctx, self._addr(segs), nseg, nstripes, self._addr(pieces),
                                          flags, self._stream(stream))
        _raise(self.scheme.ctx, rc)

    def decode_segments(self, nums: Iterable[int], piece_ptrs: Iterable[int], nstripes: int, out, nseg: int = 1,
                        piece_seg_stride: int = 0, out_seg_stride: int = 0, stream=None):
        """Decode (Correct + Rebuild) of a whole segment's pieces on the device
        (ec_decode_segments; StripeReader with error detection, stripe.go:407-408):
        corrected shares are written back into the pieces; returns when done."""
        nums = list(nums)
        ptrs = [self._addr(p) for p in piece_ptrs]
        if len(ptrs) != len(nums):
            raise ValueError("nums and piece pointers differ in length")
        c_nums = (ctypes.c_int * max(len(nums), 1))(*nums)
        c_ptrs = (ctypes.c_void_p * max(len(ptrs), 1))(*ptrs)
        rc = self._lib.ec_decode_segments_batched(self.scheme.ctx, len(nums), c_nums, c_ptrs, nstripes, nseg,
                                                  piece_seg_stride, out_seg_stride, self._addr(out),
                                                  self._stream(stream))
        _raise(self.scheme.ctx, rc)

    def rebuild_segments(self, nums: Iterable[int], piece_ptrs: Iterable[int], nstripes: int, out, nseg: int = 1,
                         piece_seg_stride: int = 0, out_seg_stride: int = 0, stream=None):
        nums = list(nums)
        ptrs = [self._addr(p) for p in piece_ptrs]
        if len(ptrs) != len(nums):
            raise ValueError("nums and piece pointers differ in length")
        c_nums = (ctypes.c_int * max(len(nums), 1))(*nums)
        c_ptrs = (ctypes.c_void_p * max(len(ptrs), 1))(*ptrs)
        rc = self._lib.ec_rebuild_segments_batched(self.scheme.ctx, len(nums), c_nums, c_ptrs, nstripes, nseg,
                                                   piece_seg_stride, out_seg_stride, self._addr(out),
                                                   self._stream(stream))
        _raise(self.scheme.ctx, rc)

    def _sets_args(self, sets, outs):
        sets = [(list(nums), [self._addr(p) for p in ptrs]) for nums, ptrs in sets]
        outs = [self._addr(o) for o in outs]
        if len(outs) != len(sets):
            raise ValueError("one output per segment")
        for nums, ptrs in sets:
            if len(nums) != len(ptrs):
                raise ValueError("nums and piece pointers differ in length")
        nseg = len(sets)
        flat_n = [x for nums, _ in sets for x in nums]
        flat_p = [x for _, ptrs in sets for x in ptrs]
        return (nseg, (ctypes.c_int * max(nseg, 1))(*[len(nums) for nums, _ in sets]),
                (ctypes.c_int * max(len(flat_n), 1))(*flat_n), (ctypes.c_void_p * max(len(flat_p), 1))(*flat_p),
                (ctypes.c_void_p * max(nseg, 1))(*outs))

    def rebuild_segments_sets(self, sets, nstripes: int, outs, stream=None):
        """Rebuild of many segments, each from a share set of its own, in one
        stream-ordered pass (ec_rebuild_segments_sets): what one StripeReader
        per download does for each segment with whichever k pieces answered
        first (stripe.go:314-354, client.go:273-308), several segments at once
        under prefetch (store.go:240-253).  Asynchronous on `stream`."""
        nseg, nsh, nums, ptrs, optr = self._sets_args(sets, outs)
        rc = self._lib.ec_rebuild_segments_sets(self.scheme.ctx, nseg, nsh, nums, ptrs, nstripes, optr,
                                                self._stream(stream))
        _raise(self.scheme.ctx, rc)

    def decode_segments_sets(self, sets, nstripes: int, outs, stream=None):
        """Decode (Correct + Rebuild) of many segments, a share set each
        (ec_decode_segments_sets); a segment with errors has its pieces
        corrected in place, as infectious corrects share.Data; returns when
        done."""
        nseg, nsh, nums, ptrs, optr = self._sets_args(sets, outs)
        rc = self._lib.ec_decode_segments_sets(self.scheme.ctx, nseg, nsh, nums, ptrs, nstripes, optr,
                                               self._stream(stream))
        _raise(self.scheme.ctx, rc)
