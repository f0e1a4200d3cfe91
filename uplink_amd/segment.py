"""Segment-level upload integration of the encoder.

Mirrors, on the engine:

  PinnedBackend           buffer.Backend / MemoryBackend   private/storage/streams/buffer/backend.go:12-120
                          (the segment buffer, swappable via Splitter.NewBackend,
                          splitter/splitter.go:87-89) -- here in pinned host memory
                          (ec_host_alloc) so the segment crosses PCIe at full DMA rate
  SegmentPieceReader      pieceReader.PieceReader          private/storage/streams/segmentupload/single.go:228-238

The reference's PieceReader(num) re-reads the whole segment through
PadReader and runs EncodeSingle once per stripe for each of the n pieces
(n readers x stripes calls, and n passes over the segment).  Here the first
request pads the segment once and encodes every parity piece of every
stripe in one engine call (ec_encode_segments_host with
EC_FLAG_PARITY_ONLY); data pieces (num < k) are the segment's own shares
(EncodeSingle copies them, rs.go:21-23) and are served from the padded
segment, so only the n - k parity pieces come back over PCIe.
"""
from __future__ import annotations

import ctypes
import io
import threading
from typing import Optional

import numpy as np

from . import _native as N
from .eestream import EEStreamError, InfectiousError, _raise

STANDARD_MAX_ENCRYPTED_SEGMENT_SIZE = 67254016  # buffer/backend.go:20


class PinnedHost:
    """A pinned host allocation (hipHostMalloc via ec_host_alloc) viewed as
    a numpy uint8 array; freed by close()."""

    def __init__(self, nbytes: int):
        self._lib = N.load()
        self.nbytes = max(int(nbytes), 1)
        self.ptr = self._lib.ec_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"ec_host_alloc({self.nbytes}) failed")
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def close(self):
        if self.ptr:
            self.array = None
            self._lib.ec_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Pool:
    """Pinned allocations are slow to make (hipHostMalloc pins pages); keep
    freed ones for reuse by size (the role of sync.Pool in backend.go:25-38)."""

    def __init__(self):
        self._mu = threading.Lock()
        self._free = {}

    def get(self, nbytes: int) -> PinnedHost:
        with self._mu:
            lst = self._free.get(max(int(nbytes), 1))
            if lst:
                return lst.pop()
        return PinnedHost(nbytes)

    def put(self, buf: PinnedHost):
        if buf.ptr:
            with self._mu:
                self._free.setdefault(buf.nbytes, []).append(buf)


pinned_pool = _Pool()


class PinnedBackend:
    """buffer.Backend (io.Writer + io.ReaderAt + io.Closer) on pinned host
    memory, like NewMemoryBackend(cap) (backend.go:42-52)."""

    def __init__(self, cap: int = STANDARD_MAX_ENCRYPTED_SEGMENT_SIZE):
        self._mem = pinned_pool.get(cap)
        self._cap = cap
        self._size = 0
        self._mu = threading.Lock()
        self._closed = False

    def write(self, b) -> int:
        with self._mu:
            if self._closed:
                raise EEStreamError("write to closed backend")
            b = memoryview(b).cast("B")
            n = len(b)
            if self._size + n > self._cap:
                raise io.UnsupportedOperation("write past the backend capacity")  # MemoryBackend: io.ErrShortWrite
            self._mem.array[self._size:self._size + n] = np.frombuffer(b, dtype=np.uint8)
            self._size += n
            return n

    def read_at(self, n: int, off: int) -> bytes:
        with self._mu:
            if self._closed:
                raise EEStreamError("read from closed backend")
            if off >= self._size:
                return b""
            return self._mem.array[off:min(off + n, self._size)].tobytes()

    def size(self) -> int:
        return self._size

    def view(self) -> np.ndarray:
        """The written bytes, zero-copy."""
        return self._mem.array[:self._size]

    def close(self):
        with self._mu:
            if not self._closed:
                self._closed = True
                pinned_pool.put(self._mem)
                self._mem = None
        return None

    def _scratch_tail(self, total: int) -> Optional[PinnedHost]:
        """The backing allocation when it can also hold `total` bytes (the
        written data plus PadReader's padding), else None."""
        return self._mem if (not self._closed and self._mem.nbytes >= total) else None


class _OwnedStream:
    """A piece stream keeps its SegmentPieceReader alive and counted: the
    reader's pinned buffers (the padded segment the data pieces are views of,
    the parity the engine writes) go back to the pool only once the reader is
    closed and every stream it handed out is closed or gone (a view
    into a pooled buffer read after another segment took it would send that
    segment's bytes)."""

    def __init__(self, owner):
        self._owner = owner

    def close(self):
        owner, self._owner = self._owner, None
        if owner is not None:
            owner._stream_closed()
        return None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _PieceStream(_OwnedStream):
    """io.ReadCloser over one piece.  `ready(end)` is called before bytes
    [.., end) are read: for a parity piece of a streamed upload it blocks
    until the stripes holding them are in host memory (ec_upload_wait)."""

    def __init__(self, src: np.ndarray, ready=None, owner=None):
        super().__init__(owner)
        self._src, self._off, self._ready = src, 0, ready

    def read(self, n: int = -1) -> bytes:
        if self._src is None:
            raise EEStreamError("read from closed piece reader")
        end = self._src.size if n is None or n < 0 else min(self._src.size, self._off + n)
        if self._ready is not None and end > self._off:
            self._ready(end)
        b = self._src[self._off:end].tobytes()
        self._off = end
        return b

    def close(self):
        self._src = None
        return super().close()


class _DataPieceStream(_OwnedStream):
    """A data piece (num < k) is share num of every stripe of the padded
    segment (EncodeSingle copies it, rs.go:21-23): gathered per read from the
    host segment, with no engine call and nothing to wait for."""

    def __init__(self, padded: np.ndarray, num: int, owner=None):
        super().__init__(owner)
        self._p, self._num, self._off = padded, num, 0  # padded: [stripes][k][ess]
        self._size = padded.shape[0] * padded.shape[2]

    def read(self, n: int = -1) -> bytes:
        if self._p is None:
            raise EEStreamError("read from closed piece reader")
        end = self._size if n is None or n < 0 else min(self._size, self._off + n)
        if end <= self._off:
            return b""
        ess = self._p.shape[2]
        s0, s1 = self._off // ess, (end + ess - 1) // ess
        b = self._p[s0:s1, self._num, :].reshape(-1)[self._off - s0 * ess:end - s0 * ess].tobytes()
        self._off = end
        return b

    def close(self):
        self._p = None
        return super().close()


class SegmentPieceReader:
    """pieceReader (single.go:228-238): piece_reader(num) streams piece num
    of the segment (PadReader to the stripe size, then EncodeSingle per
    stripe).  The first call pads the segment once and starts one streamed
    engine call for every parity piece (ec_upload_begin): the segment goes
    through the GPU in chunks of stripes, and a parity piece's reader blocks
    only until the chunk holding the bytes it is asked for has arrived, so an
    upload starts after the first chunk, as the reference's per-stripe
    EncodedReader does (segmentupload/encode.go:39-75).  With hash_pieces the
    same streamed call also hashes every piece chunk by chunk
    (EC_FLAG_HASH_PIECES), as the reference hashes each piece through a
    TeeReader while it streams (piecestore/upload.go:155,262-270):
    piece_hash(num) waits only for the tree fold after the last chunk."""

    def __init__(self, segment, redundancy, hash_pieces: bool = False, chunk_stripes: int = 0):
        self.segment = segment  # bytes-like, numpy array, or PinnedBackend
        self.redundancy = redundancy
        self.hash_pieces = hash_pieces  # also compute every piece's BLAKE3 in the same engine call
        self.chunk_stripes = chunk_stripes  # streamed upload chunk (0: the library's growing chunks)
        self._mu = threading.RLock()  # (re-entered when a stream's __del__ runs under it)
        self._padded: Optional[np.ndarray] = None
        self._parity: Optional[PinnedHost] = None
        self._hashes: Optional[np.ndarray] = None
        self._upload = None  # ec_upload handle of the streamed encode
        self._bufs = []
        self._streams = 0  # piece streams handed out and not yet closed
        self._closing = False
        self.stripes = 0

    def _prepare(self):
        with self._mu:
            # after close() nothing may be allocated or begun again (the buffers went back to
            # the pool; a new upload would only be reclaimed by __del__)
            if self._closing:
                raise EEStreamError("piece reader used after close")
            if self._padded is not None:
                return
            rs = self.redundancy
            k, n, ess = rs.required_count(), rs.total_count(), rs.erasure_share_size()
            stripe = rs.stripe_size()
            data = self.segment.view() if isinstance(self.segment, PinnedBackend) else np.frombuffer(
                memoryview(self.segment).cast("B"), dtype=np.uint8)
            size = data.size
            # PadReader: p = 4 + (stripe - (size+4) % stripe) % stripe bytes
            p = 4 + (stripe - (size + 4) % stripe) % stripe
            stripes = (size + p) // stripe
            own = self.segment._scratch_tail(size + p) if isinstance(self.segment, PinnedBackend) else None
            if own is not None:  # pad in place, right after the segment in its own pinned buffer
                padded = own
            else:
                padded = pinned_pool.get(stripes * stripe)
                padded.array[:size] = data
                self._bufs.append(padded)
            padded.array[size:size + p] = p & 0xFF
            padded.array[size + p - 4:size + p] = np.frombuffer(p.to_bytes(4, "big"), dtype=np.uint8)
            parity = pinned_pool.get((n - k) * stripes * ess)
            self._bufs.append(parity)
            ctx = rs.scheme.ctx if hasattr(rs, "scheme") else rs.ctx
            if self.hash_pieces and n == k:  # no parity to stream: hash the data pieces in one call
                self._hashes = np.empty((n, 32), dtype=np.uint8)
                rc = N.load().ec_encode_segments_host_hashed(ctx, padded.ptr, 1, stripes, parity.ptr,
                                                             self._hashes.ctypes.data, N.EC_FLAG_PARITY_ONLY)
                _raise(None, rc)
            elif n > k:
                # parity streamed chunk by chunk; with hash_pieces the BLAKE3 of all n pieces along
                # with it (piecestore/upload.go:155,270)
                h = ctypes.c_void_p()
                flags = N.EC_FLAG_PARITY_ONLY | (N.EC_FLAG_HASH_PIECES if self.hash_pieces else 0)
                rc = N.load().ec_upload_begin(ctx, padded.ptr, stripes, parity.ptr, flags, self.chunk_stripes,
                                              ctypes.byref(h))
                _raise(None, rc)
                self._upload = h
            self.stripes = stripes
            self._padded = padded.array[:stripes * stripe].reshape(stripes, k, ess)
            self._parity = parity.array[:(n - k) * stripes * ess].reshape(n - k, stripes * ess)

    def piece_reader(self, num: int):
        rs = self.redundancy
        k, n = rs.required_count(), rs.total_count()
        if num < 0:  # infectious EncodeSingle's errors (segmentupload/encode_test.go:53,63)
            raise InfectiousError("num must be non-negative")
        if num >= n:
            raise InfectiousError(f"num must be less than {n}")
        self._prepare()
        with self._mu:
            if self._closing or self._padded is None:
                raise EEStreamError("piece reader used after close")
            self._streams += 1
            if num < k:  # EncodeSingle of a data share is the share itself (rs.go:21-23)
                return _DataPieceStream(self._padded, num, owner=self)
            return _PieceStream(self._parity[num - k], self._wait if self._upload is not None else None, owner=self)

    def _stream_closed(self):
        with self._mu:
            self._streams -= 1
            if not (self._closing and self._streams == 0):
                return
            rc = self._release_locked()
        _raise(None, rc)

    def _wait(self, end: int):
        """Block until bytes [0, end) of every parity piece are in host memory
        (a stream being read holds the reader open: the handle stays valid)."""
        ess = self.redundancy.erasure_share_size()
        h = self._upload
        if h is None:
            raise EEStreamError("piece reader used after close")
        _raise(None, N.load().ec_upload_wait(h, (end + ess - 1) // ess))

    def ready_stripes(self) -> int:
        """Leading stripes of every parity piece already in host memory (no wait)."""
        if self._upload is None:
            return self.stripes if self._padded is not None else 0
        return int(N.load().ec_upload_ready(self._upload))

    def piece_hash(self, num: int) -> bytes:
        """BLAKE3-256 of piece num: what the piecestore upload of that piece
        sends as PieceHash.Hash (upload.go:270).  Needs hash_pieces=True."""
        if not self.hash_pieces:
            raise EEStreamError("piece hashes were not requested (hash_pieces=False)")
        if not 0 <= num < self.redundancy.total_count():
            raise InfectiousError(f"num must be less than {self.redundancy.total_count()}")
        self._prepare()
        with self._mu:
            if self._hashes is None:
                if self._upload is None:
                    raise EEStreamError("piece reader used after close")
                hashes = np.empty((self.redundancy.total_count(), 32), dtype=np.uint8)
                _raise(None, N.load().ec_upload_hashes(self._upload, hashes.ctypes.data))
                self._hashes = hashes
            return self._hashes[num].tobytes()

    def _release_locked(self) -> int:
        """End the engine call and return the buffers to the pool (under _mu)."""
        rc = 0
        if self._upload is not None:  # the engine may still be writing the parity buffer
            rc = N.load().ec_upload_end(self._upload)
            self._upload = None
        for b in self._bufs:
            pinned_pool.put(b)
        self._bufs = []
        self._padded = self._parity = self._hashes = None
        return rc

    def close(self):
        """Close the reader; its buffers go back to the pool once every piece
        stream it handed out is closed too (streams still being read keep them)."""
        with self._mu:
            self._closing = True
            if self._streams > 0:
                return None
            rc = self._release_locked()
        _raise(None, rc)

    def __del__(self):
        # unreachable, and so is every stream it handed out (each holds the reader): nothing can
        # read its buffers any more
        try:
            with self._mu:
                self._closing = True
                self._streams = 0
                self._release_locked()
        except Exception:
            pass
