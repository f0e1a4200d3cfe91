"""Host-side mirror of storj/uplink's eestream stream layer, driving the
MI355X engine with batched calls (§8f rows 1-2).

Same names, argument meaning and error behaviour as the Go reference:

  encode_reader2 / EncodedPiece   EncodeReader2          private/eestream/encode.go:101-208
  EncodedRanger                   NewEncodedRanger/Range private/eestream/encode.go:213-268
  StripeReader / read_stripes     NewStripeReader / ReadStripes
                                                         private/eestream/stripe.go:43-444
  decode_readers2 / DecodedReader DecodeReaders2         private/eestream/decode.go:20-144
  decode / DecodedRanger          Decode                 private/eestream/decode.go:146-227
  calc_encompassing_blocks        encryption.CalcEncompassingBlocks (storj.io/common)
  fatal_read_closer / limit_read_closer / nop_closer     storj.io/common/readcloser

What differs from the reference is only where the arithmetic happens:

  * encode: the per-piece EncodeSingle per stripe (encode.go:187) becomes one
    batched encode of `batch_stripes` stripes for all n pieces at once
    (scheme.encode_stripes -> ec_encode_segments_host); piece readers then
    serve their share bytes from that batch.
  * decode: ReadStripes' per-stripe Rebuild (stripe.go:407-413) becomes one
    batched rebuild of every stripe found ready (scheme.rebuild_stripes ->
    ec_rebuild_segments_host: one share choice and one inversion per ready
    set).  With error detection the run goes through one Decode (Correct +
    Rebuild, Berlekamp-Welch on the flagged byte columns) instead of one per
    stripe: a column that cannot be corrected fails the run, and ReadStripes
    then asks for one more share and starts over, as the reference does for
    a failing stripe (stripe.go:419-424).

A reader here is any object with read(n) -> bytes (b"" at end of stream,
an exception on error) and close().  The scheme is an RSScheme (GPU); tests
may pass another object with the same methods.
"""
from __future__ import annotations

import io
import threading
import time
from typing import Dict, List, Optional

import numpy as np

from .eestream import EEStreamError, InfectiousError, NotEnoughShares, Share, TooManyErrors

MAX_STRIPES_AHEAD = 256          # stripe.go:26
INACTIVE_CHECK_INTERVAL = 1.0    # stripe.go:27 (seconds)
INACTIVE_CHECK_MAX_COUNT = 5     # stripe.go:28
GLOBAL_BUF_SIZE = 32 * 1024      # bufpool.go:13 (decode.go:60 out buffer)


class ErrInactive(EEStreamError):
    """eestream.ErrInactive (common.go:18): errs.Class("quiescence")."""

    def __init__(self, msg: str = ""):
        Exception.__init__(self, "quiescence" + (": " + msg if msg else ""))


class UnexpectedEOF(EOFError):
    def __init__(self):
        super().__init__("unexpected EOF")


def _is_eof(e: BaseException) -> bool:
    return isinstance(e, EOFError) and not isinstance(e, UnexpectedEOF)


# ------------------------------------------------------------------ readcloser
class _Fatal:
    def __init__(self, err: BaseException):
        self._err = err

    def read(self, n: int = -1) -> bytes:
        raise self._err

    def close(self):
        return None


def fatal_read_closer(err: BaseException):
    """readcloser.FatalReadCloser: every Read returns err, Close succeeds."""
    return _Fatal(err)


class _Limit:
    def __init__(self, r, n: int):
        self._r, self._left = r, n

    def read(self, n: int = -1) -> bytes:
        if self._left <= 0:
            return b""
        want = self._left if n is None or n < 0 else min(n, self._left)
        b = self._r.read(want)
        self._left -= len(b)
        return b

    def close(self):
        c = getattr(self._r, "close", None)
        return c() if c else None


def limit_read_closer(r, n: int):
    """readcloser.LimitReadCloser: at most n bytes, Close closes r."""
    return _Limit(r, n)


class _Nop:
    def __init__(self, r):
        self._r = r

    def read(self, n: int = -1) -> bytes:
        return self._r.read(n)

    def close(self):
        return None


def nop_closer(r):
    """io.NopCloser."""
    return _Nop(r)


def read_all(r) -> bytes:
    """io.ReadAll."""
    out = bytearray()
    while True:
        b = r.read(1 << 20)
        if not b:
            return bytes(out)
        out += b


def read_full(r, n: int) -> bytes:
    """io.ReadFull: UnexpectedEOF when the stream ends early (EOFError when
    it is empty)."""
    out = bytearray()
    while len(out) < n:
        b = r.read(n - len(out))
        if not b:
            if not out:
                raise EOFError("EOF")
            raise UnexpectedEOF()
        out += b
    return bytes(out)


def calc_encompassing_blocks(offset: int, length: int, block_size: int):
    """encryption.CalcEncompassingBlocks: the blocks covering [offset, offset+length)."""
    first = offset // block_size
    if length <= 0:
        return first, 0
    last = (offset + length) // block_size
    if (offset + length) % block_size == 0:
        return first, last - first
    return first, last - first + 1


# ------------------------------------------------------------------ encode
class _BatchEncoder:
    """The shared half of EncodeReader2: reads the source a batch of stripes
    at a time and encodes all n shares of the batch in one engine call.  A
    batch is kept until every piece reader has moved past it (the role of the
    tee in encode.go:118-131)."""

    def __init__(self, r, rs, batch_stripes: int):
        self._r = r
        self._rs = rs
        self._stripe = rs.stripe_size()
        self._batch = max(1, batch_stripes)
        self._mu = threading.Lock()
        self._batches: Dict[int, np.ndarray] = {}  # index -> [n][stripes*ess]
        self._err: Optional[BaseException] = None
        self._end: Optional[int] = None  # index of the first batch past the end
        self._next = 0
        self._pos = [0] * rs.total_count()  # next batch each piece needs

    def batch(self, idx: int) -> Optional[np.ndarray]:
        """shares [n][m*ess] of batch idx, None past the end; raises the
        source error (or UnexpectedEOF for a partial stripe) at its batch."""
        with self._mu:
            while idx >= self._next and self._end is None:
                self._encode_next()
            if idx in self._batches:
                return self._batches[idx]
            if self._err is not None:
                raise self._err
            return None

    def _encode_next(self):
        want = self._batch * self._stripe
        buf = bytearray()
        try:
            while len(buf) < want:
                b = self._r.read(want - len(buf))
                if not b:
                    break
                buf += b
        except BaseException as e:  # source error: every piece sees it
            self._err = e
            self._end = self._next
            return
        m, rem = divmod(len(buf), self._stripe)
        if m:
            data = np.frombuffer(bytes(buf[:m * self._stripe]), dtype=np.uint8)
            self._batches[self._next] = self._rs.encode_stripes(data)
            self._next += 1
        if rem or m < self._batch:
            self._end = self._next
            if rem:
                self._err = UnexpectedEOF()  # io.ReadFull of a partial stripe (encode.go:180)

    def advance(self, num: int, idx: int):
        with self._mu:
            self._pos[num] = idx
            low = min(self._pos)
            for b in [b for b in self._batches if b < low]:
                del self._batches[b]


class EncodedPiece:
    """encodedPiece (encode.go:161-208): the stream of erasure share `num`."""

    def __init__(self, enc: _BatchEncoder, num: int):
        self._enc, self.num = enc, num
        self._batch_idx = 0
        self._cur: Optional[np.ndarray] = None
        self._off = 0
        self._err: Optional[BaseException] = None
        self._closed = False

    def read(self, n: int = -1) -> bytes:
        if self._err is not None:
            raise self._err
        want = (1 << 62) if n is None or n < 0 else n
        out = bytearray()
        while len(out) < want:
            if self._cur is None or self._off >= self._cur.size:
                try:
                    shares = self._enc.batch(self._batch_idx)
                except BaseException as e:
                    self._err = e
                    if out:
                        break
                    raise
                if shares is None:
                    break
                self._cur = shares[self.num]
                self._off = 0
                self._batch_idx += 1
                self._enc.advance(self.num, self._batch_idx - 1)
            take = min(self._cur.size - self._off, want - len(out))
            out += self._cur[self._off:self._off + take].tobytes()
            self._off += take
        return bytes(out)

    def close(self):
        if not self._closed:
            self._closed = True
            self._enc.advance(self.num, 1 << 62)
        return None


def encode_reader2(r, rs, batch_stripes: int = 256) -> List[EncodedPiece]:
    """EncodeReader2 (encode.go:106-148): n piece readers over the stream r,
    which must end on a stripe boundary (PadReader output)."""
    enc = _BatchEncoder(r, rs, batch_stripes)
    return [EncodedPiece(enc, i) for i in range(rs.total_count())]


class ByteRanger:
    """ranger.ByteRanger."""

    def __init__(self, data: bytes):
        self._d = bytes(data)

    def size(self) -> int:
        return len(self._d)

    def range(self, offset: int, length: int):
        if offset < 0:
            raise EEStreamError("negative offset")
        if length < 0:
            raise EEStreamError("negative length")
        if offset + length > len(self._d):
            raise EEStreamError("buffer runoff")
        return nop_closer(io.BytesIO(self._d[offset:offset + length]))


class EncodedRanger:
    """EncodedRanger (encode.go:213-268)."""

    def __init__(self, rr, rs):
        if rr.size() % rs.stripe_size():
            raise EEStreamError("invalid erasure encoder and range reader combo. range reader size must be a "
                                "multiple of erasure encoder block size")
        self.rr, self.rs = rr, rs

    def output_size(self) -> int:
        return self.rr.size() // self.rs.stripe_size() * self.rs.erasure_share_size()

    def range(self, offset: int, length: int):
        ess, stripe = self.rs.erasure_share_size(), self.rs.stripe_size()
        first, count = calc_encompassing_blocks(offset, length, ess)
        r = self.rr.range(first * stripe, count * stripe)
        out = []
        for rd in encode_reader2(r, self.rs):
            skip = offset - first * ess
            if skip and len(rd.read(skip)) != skip:
                raise EEStreamError(str(UnexpectedEOF()))
            out.append(limit_read_closer(rd, length))
        return out


def new_encoded_ranger(rr, rs) -> EncodedRanger:
    return EncodedRanger(rr, rs)


# ------------------------------------------------------------------ decode
class _Piece:
    """pieceReader + StreamingPiece (stripe.go:31-40, piece.go): one share
    stream read by its own thread into a buffer of whole shares."""

    def __init__(self, num: int, source, total_size: int, ess: int):
        self.num = num
        self.source = source
        self.left = total_size
        self.ess = ess
        self.buf = np.zeros(max(total_size, 1), dtype=np.uint8)
        self.received = 0       # bytes
        self.shares = 0         # whole shares received (the bundy watermark)
        self.err: Optional[BaseException] = None
        self.completed = 0      # stripes the core has consumed (backpressure)


class StripeReader:
    """StripeReader (stripe.go:43-444): reads the piece streams in parallel
    and returns decoded stripes; see the module notes for the batching."""

    def __init__(self, readers: Dict[int, object], scheme, total_stripes: int, error_detection: bool):
        ess = scheme.erasure_share_size()
        total = total_stripes * ess
        self.scheme = scheme
        self.total_stripes = total_stripes
        self.error_detection = error_detection
        self.pieces = [_Piece(num, src, total, ess) for num, src in readers.items()]
        minimum = scheme.required_count()
        if error_detection and minimum < len(self.pieces):
            minimum += 1
        self.needed = minimum
        self.returned = 0
        self._cv = threading.Condition()
        self._running = len(self.pieces)
        self._inactive = False
        self._closed = False
        self._threads = [threading.Thread(target=self._read_shares, args=(p,), daemon=True) for p in self.pieces]
        for t in self._threads:
            t.start()
        self._watch = threading.Thread(target=self._watchdog, daemon=True)
        self._watch.start()

    # -- stripe.go:165-211
    def _read_shares(self, p: _Piece):
        try:
            while p.left > 0:
                n = min(p.left, max(p.ess, 1 << 16))
                try:
                    b = p.source.read(n)
                except BaseException as e:  # a read error ends this piece
                    if not _is_eof(e):
                        p.err = e
                    break
                if not b:
                    break
                b = b[:p.left]
                p.buf[p.received:p.received + len(b)] = np.frombuffer(b, dtype=np.uint8)
                p.received += len(b)
                p.left -= len(b)
                with self._cv:
                    p.shares = p.received // p.ess
                    self._cv.notify_all()
                    while (p.shares > p.completed + MAX_STRIPES_AHEAD and p.completed < self.total_stripes
                           and not self._closed):
                        self._cv.wait()
        finally:
            with self._cv:
                self._running -= 1
                self._cv.notify_all()

    # -- stripe.go:125-160: no progress for INACTIVE_CHECK_MAX_COUNT checks
    def _watchdog(self):
        last, same = None, 0
        while True:
            time.sleep(INACTIVE_CHECK_INTERVAL)
            with self._cv:
                if self._running == 0 or self._closed:
                    return
                snap = tuple(p.shares for p in self.pieces)
                if snap != last:
                    last, same = snap, 0
                    continue
                same += 1
                if same == INACTIVE_CHECK_MAX_COUNT:
                    self._inactive = True
                    self._cv.notify_all()
                    return

    def _combine_errs(self) -> EEStreamError:
        errs = [f"error retrieving piece {p.num:02d}: {p.err}" for p in self.pieces if p.err is not None]
        if errs:
            return EEStreamError("; ".join(errs))
        return EEStreamError("programmer error: no errors to combine")

    def read_stripes(self, next_stripe: int, out_cap: int = GLOBAL_BUF_SIZE):
        """ReadStripes (stripe.go:275-444): (bytes of >= 1 stripes, count)."""
        if next_stripe != self.returned:
            raise EEStreamError("unexpected next stripe")
        stripe_size = self.scheme.stripe_size()
        if out_cap <= 0:
            out_cap = GLOBAL_BUF_SIZE
        max_stripes = out_cap // stripe_size
        if self.returned + max_stripes > self.total_stripes:
            max_stripes = self.total_stripes - self.returned
        if max_stripes <= 0:
            raise EOFError("EOF")
        required = self.returned + 1
        while True:
            with self._cv:
                while True:
                    if self._inactive:
                        raise ErrInactive()
                    found = self.returned + max_stripes
                    ready = []
                    for p in self.pieces:
                        if p.shares >= required:
                            ready.append(p)
                            found = min(found, p.shares)
                    if len(ready) >= self.needed:
                        break
                    if self._running + len(ready) < self.needed:
                        raise self._combine_errs()
                    self._cv.wait(timeout=INACTIVE_CHECK_INTERVAL)
            try:
                data = self._decode_range(ready, self.returned, found)
            except (NotEnoughShares, TooManyErrors) as e:
                with self._cv:
                    if self.needed < len(self.pieces):  # bundy.IncreaseNeededShares: start over
                        self.needed += 1
                        continue
                raise EEStreamError(f"error decoding data: {e}")
            except InfectiousError as e:
                raise EEStreamError(f"error decoding data: {e}")
            with self._cv:
                for p in self.pieces:
                    p.completed = max(p.completed, found)
                self._cv.notify_all()
            count = found - self.returned
            self.returned = found
            return data, count

    def _decode_range(self, ready: List[_Piece], lo: int, hi: int) -> bytes:
        ess = self.scheme.erasure_share_size()
        if not self.error_detection:
            views = [p.buf[lo * ess:hi * ess] for p in ready]
            return self.scheme.rebuild_stripes([p.num for p in ready], views, hi - lo).tobytes()
        # Reed-Solomon is column-independent, so the run's bytes of each piece
        # form one long share: a single Decode (Correct + Rebuild) covers every
        # stripe of the run; its [k][run*ess] output is re-laid stripe-major.
        k, m = self.scheme.required_count(), hi - lo
        shares = [Share(p.num, p.buf[lo * ess:hi * ess].copy()) for p in ready]
        out = self.scheme.decode(None, shares)
        return np.ascontiguousarray(out[:k * m * ess].reshape(k, m, ess).transpose(1, 0, 2)).tobytes()

    def close(self):
        """Close (stripe.go:230-240): release the piece threads; does not
        close the source readers."""
        with self._cv:
            self._closed = True
            for p in self.pieces:
                p.completed = self.total_stripes
            self._cv.notify_all()
        return None


def new_stripe_reader(readers, scheme, total_stripes: int, error_detection: bool) -> StripeReader:
    return StripeReader(readers, scheme, total_stripes, error_detection)


class DecodedReader:
    """decodedReader (decode.go:20-144)."""

    def __init__(self, readers, es, expected_stripes: int, out_cap: int, force_error_detection: bool):
        self.readers = readers
        self.scheme = es
        self.expected = expected_stripes
        self.out_cap = out_cap
        self.current = 0
        self._buf = b""
        self._err: Optional[BaseException] = None
        self.stripe_reader = StripeReader(readers, es, expected_stripes, force_error_detection)
        self._closed = False

    def read(self, n: int = -1) -> bytes:
        if not self._buf:
            if self._err is not None:
                if _is_eof(self._err):
                    return b""
                raise self._err
            if self.current >= self.expected:
                self._err = EOFError("EOF")
                return b""
            try:
                self._buf, count = self.stripe_reader.read_stripes(self.current, self.out_cap)
            except BaseException as e:
                self._err = e
                if _is_eof(e):
                    return b""
                raise
            self.current += count
        take = len(self._buf) if n is None or n < 0 else min(n, len(self._buf))
        b, self._buf = self._buf[:take], self._buf[take:]
        return b

    def close(self):
        """Close (decode.go:103-139): closes every piece reader and the stripe
        reader; errors only when more readers failed to close than the scheme
        can lose."""
        if self._closed:
            return None
        self._closed = True
        errs = []
        for r in self.readers.values():
            try:
                c = getattr(r, "close", None)
                if c:
                    c()
            except BaseException as e:
                errs.append(e)
        self.stripe_reader.close()
        if len(self.readers) - self.scheme.required_count() - len(errs) < 0:
            raise EEStreamError("; ".join(str(e) for e in errs))
        return None


def decode_readers2(rs: Dict[int, object], es, expected_size: int, mbm: int = 0,
                    force_error_detection: bool = False, out_buffer: int = GLOBAL_BUF_SIZE):
    """DecodeReaders2 (decode.go:44-78).  out_buffer is the ReadStripes output
    capacity (the reference's 32 KiB outbufmem, decode.go:60); a larger one
    lets each ReadStripes decode more stripes in one engine call (§8f row 2)."""
    if expected_size < 0:
        return fatal_read_closer(EEStreamError("negative expected size"))
    if expected_size % es.stripe_size():
        return fatal_read_closer(EEStreamError(
            f"expected size ({expected_size}) not a factor decoded block size ({es.stripe_size()})"))
    if mbm < 0:
        return fatal_read_closer(EEStreamError("negative max buffer memory"))
    return DecodedReader(rs, es, expected_size // es.stripe_size(), out_buffer, force_error_detection)


class DecodedRanger:
    """decodedRanger (decode.go:146-213)."""

    def __init__(self, es, rrs, in_size: int, mbm: int, force: bool):
        self.es, self.rrs, self.in_size, self.mbm, self.force = es, rrs, in_size, mbm, force

    def size(self) -> int:
        return self.in_size // self.es.erasure_share_size() * self.es.stripe_size()

    def range(self, offset: int, length: int):
        ess, stripe = self.es.erasure_share_size(), self.es.stripe_size()
        first, count = calc_encompassing_blocks(offset, length, stripe)
        readers = {}
        for i, rr in self.rrs.items():
            try:
                readers[i] = rr.range(first * ess, count * ess)
            except BaseException as e:
                readers[i] = fatal_read_closer(e)
        r = decode_readers2(readers, self.es, count * stripe, self.mbm, self.force)
        skip = offset - first * stripe
        while skip > 0:
            b = r.read(skip)
            if not b:
                raise EEStreamError("EOF")
            skip -= len(b)
        return limit_read_closer(r, length)


def decode(rrs: Dict[int, object], es, mbm: int = 0, force_error_detection: bool = False):
    """Decode (decode.go:154-191): a Ranger over the decoded stream."""
    if mbm < 0:
        raise EEStreamError("negative max buffer memory")
    if len(rrs) < es.required_count():
        raise EEStreamError("not enough readers to reconstruct data!")
    size = -1
    for rr in rrs.values():
        if size == -1:
            size = rr.size()
        elif size != rr.size():
            raise EEStreamError("decode failure: range reader sizes don't all match")
    if size == -1:
        return ByteRanger(b"")
    if size % es.erasure_share_size():
        raise EEStreamError("invalid erasure decoder and range reader combo. range reader size "
                            f"({size}) must be a multiple of erasure encoder block size ({es.erasure_share_size()})")
    return DecodedRanger(es, rrs, size, mbm, force_error_detection)
