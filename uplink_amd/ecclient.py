"""Host mirror of storj/uplink's private/ecclient: the
piece fan-out of an upload (`put` / `PutSingleResult`, client.go:77-209) and
the download-side sizing of `GetWithOptions` (client.go:273-308) over the
GPU engine.

What the GPU does and what stays on the host:
  * put: the padded segment is encoded by one batched engine call per run of
    stripes (streams.encode_reader2 -> ec_encode_segments), not n goroutines
    each running EncodeSingle per stripe; the n piece readers are then handed
    to one putter thread each, exactly as client.go:141-146 starts one
    goroutine per piece, with the reference's long-tail cut (cancel the rest
    once OptimalThreshold pieces are stored, client.go:178-181) and its
    threshold errors.
  * GetWithOptions: paddedSize = calcPadded(size, stripe) (client.go:284,
    333-339), pieceSize = paddedSize / k (:285), one lazy ranger per non-nil
    limit (:287-298, :341-471), eestream.Decode (streams.decode: one engine
    rebuild per ready run of stripes) and encryption.Unpad(rr, paddedSize -
    size) (:306).

The network side -- dialing storage nodes, piecestore upload/download, order
limits and signatures -- is out of scope: a `PieceStore` object
stands in for it with two calls, put_piece(limit, reader, cancel) and
download(limit, offset, length) (the loopback-piecestore pattern of
private/piecestore/client_test.go:76-179).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from . import eestream, streams

__all__ = ["ECClientError", "AddressedOrderLimit", "calc_padded", "unique", "non_nil_count", "ECClient",
           "SubRanger", "unpad", "LazyPieceRanger", "PieceUploadResult"]


class ECClientError(Exception):
    """errs.Class("ecclient") (private/ecclient/common.go:11)."""

    def __init__(self, msg: str, cause: Optional[BaseException] = None):
        super().__init__("ecclient: " + msg)
        self.cause = cause


class Canceled(Exception):
    """context.Canceled, as PutPiece reports a piece cut by the long-tail cancel."""


@dataclass(frozen=True)
class AddressedOrderLimit:
    """The parts of pb.AddressedOrderLimit the fan-out reads: the storage
    node id (limit.GetLimit().StorageNodeId) and its address."""
    node_id: bytes
    address: str = ""
    piece_id: int = 0


@dataclass
class PieceUploadResult:
    """pb.SegmentPieceUploadResult (client.go:89-93)."""
    piece_num: int
    node_id: bytes
    hash: object


def calc_padded(size: int, block_size: int) -> int:
    """calcPadded (client.go:333-339): size rounded up to whole stripes."""
    mod = size % block_size
    return size if mod == 0 else size + block_size - mod


def non_nil_count(limits: Sequence[Optional[AddressedOrderLimit]]) -> int:
    """nonNilCount (private/ecclient/common.go)."""
    return sum(1 for x in limits if x is not None)


def unique(limits: Optional[Sequence[Optional[AddressedOrderLimit]]]) -> bool:
    """unique (client.go:310-331): no node twice; nil limits are ignored."""
    if not limits or len(limits) < 2:
        return True
    ids = sorted(x.node_id if x is not None else b"" for x in limits)
    return not any(ids[i] and ids[i] == ids[i - 1] for i in range(1, len(ids)))


class SubRanger:
    """ranger.Subrange: the first `length` bytes of `rr` from `offset`."""

    def __init__(self, rr, offset: int, length: int):
        if offset < 0 or length < 0 or offset + length > rr.size():
            raise ECClientError("invalid subrange")
        self.rr, self.offset, self.length = rr, offset, length

    def size(self) -> int:
        return self.length

    def range(self, offset: int, length: int):
        if offset < 0 or length < 0 or offset + length > self.length:
            raise ECClientError("range beyond end")
        return self.rr.range(self.offset + offset, length)


def unpad(rr, padding: int) -> SubRanger:
    """encryption.Unpad(rr, padding) (storj.io/common): the ranger without its
    last `padding` bytes (the download side knows the size, so no trailer)."""
    return SubRanger(rr, 0, rr.size() - padding)


class LazyPieceRanger:
    """lazyPieceRanger (client.go:341-471): a piece of known size whose bytes
    are fetched from the node only when a range is read."""

    def __init__(self, store, limit: AddressedOrderLimit, size: int):
        self.store, self.limit, self._size = store, limit, size

    def size(self) -> int:
        return self._size

    def range(self, offset: int, length: int):
        return _LazyPieceReader(self, offset, length)


class _LazyPieceReader:
    """lazyPieceReader: dials (here: asks the store) on the first Read."""

    def __init__(self, ranger: LazyPieceRanger, offset: int, length: int):
        self.ranger, self.offset, self.length = ranger, offset, length
        self._mu = threading.Lock()
        self._r = None
        self._closed = False

    def read(self, n: int = -1) -> bytes:
        with self._mu:
            if self._closed:
                return b""
            if self._r is None:
                self._r = self.ranger.store.download(self.ranger.limit, self.offset, self.length)
            r = self._r
        return r.read(n)

    def close(self):
        with self._mu:
            if self._closed:
                return
            self._closed = True
            if self._r is not None and hasattr(self._r, "close"):
                self._r.close()


class ECClient:
    """ecclient.Client (client.go:36-44) over a PieceStore stand-in."""

    def __init__(self, store, memory_limit: int = 0):
        self.store = store
        self.memory_limit = memory_limit
        self.force_error_detection = False

    def with_force_error_detection(self, force: bool) -> "ECClient":
        self.force_error_detection = force
        return self

    # ------------------------------------------------------------- upload
    def put_piece(self, limit: Optional[AddressedOrderLimit], reader, cancel: threading.Event,
                  parent: Optional[threading.Event] = None):
        """PutPiece (client.go:211-256): a nil limit drains its reader; the
        store's error is wrapped like the reference wraps the upload error.
        `cancel` is the pieces context (canceled by the long-tail cut or with
        its parent), `parent` the caller's context."""
        try:
            if limit is None:
                streams.read_all(reader)
                return None
            try:
                return self.store.put_piece(limit, reader, cancel)
            except Exception as e:  # noqa: BLE001 - the reference wraps every upload error
                user = parent is not None and parent.is_set()
                if cancel.is_set() or user:
                    # client.go:232-243: once the pieces context is canceled, whatever the store
                    # returned is a cancel -- by the user when the parent context is canceled, else
                    # the long-tail cut -- with context.Canceled the primary error of the chain
                    cause = e if isinstance(e, Canceled) else Canceled(f"context canceled: {e}")
                    if user:
                        raise ECClientError(f"upload canceled by user: {e}", cause)
                    raise ECClientError(f"upload cut due to slow connection (node:{limit.node_id.hex()}): {e}", cause)
                raise ECClientError(f"upload failed (node:{limit.node_id.hex()}, address:{limit.address}): {e}", e)
        finally:
            if hasattr(reader, "close"):
                reader.close()

    def put(self, limits: List[Optional[AddressedOrderLimit]], rs: eestream.RedundancyStrategy,
            data, parent: Optional[threading.Event] = None) -> Tuple[List[Optional[dict]], List[object]]:
        """put (client.go:103-209): returns (successful nodes, hashes) indexed
        by piece number, None where a piece was not stored.  `parent` is the
        caller's context: setting it cancels every upload in flight, which
        then fail as "upload canceled by user"."""
        piece_count = len(limits)
        if piece_count != rs.total_count():
            raise ECClientError(f"size of limits slice ({piece_count}) does not match total count "
                                f"({rs.total_count()}) of erasure scheme")
        nn = non_nil_count(limits)
        if nn <= rs.repair_threshold() and nn < rs.optimal_threshold():
            raise ECClientError(f"number of non-nil limits ({nn}) is less than or equal to the repair threshold "
                                f"({rs.repair_threshold()}) of erasure scheme")
        if not unique(limits):
            raise ECClientError("duplicated nodes are not allowed")
        raw = data.read() if hasattr(data, "read") else bytes(data)
        padded = eestream.pad(raw, rs.stripe_size())  # encryption.PadReader (client.go:125)
        readers = streams.encode_reader2(streams.nop_closer(_BytesReader(padded)), rs)  # EncodeReader2 (:126)

        cancel = threading.Event()  # piecesCtx / piecesCancel (:139-140)
        done = threading.Event()  # set on every way out of put (the watcher stops with it)
        try:
            return self._put_pieces(limits, rs, readers, cancel, parent, done, piece_count)
        finally:
            done.set()

    def _put_pieces(self, limits, rs, readers, cancel, parent, done, piece_count):
        infos: List[Tuple[int, Optional[BaseException], object]] = []
        cv = threading.Condition()
        if parent is not None:
            def watch():  # piecesCtx is a child of the caller's context (client.go:139)
                while not done.is_set():
                    if parent.wait(0.02):
                        cancel.set()
                        return
            threading.Thread(target=watch, daemon=True).start()

        def one(i: int):
            try:
                h = self.put_piece(limits[i], readers[i], cancel, parent)
                res = (i, None, h)
            except BaseException as e:  # noqa: BLE001 - collected like the info channel
                res = (i, e, None)
            with cv:
                infos.append(res)
                cv.notify()

        threads = [threading.Thread(target=one, args=(i,), daemon=True) for i in range(piece_count)]
        for t in threads:
            t.start()
        nodes: List[Optional[dict]] = [None] * piece_count
        hashes: List[object] = [None] * piece_count
        successful = failed = canceled = 0
        errors: List[BaseException] = []
        for _ in range(piece_count):
            with cv:
                while not infos:
                    cv.wait()
                i, err, h = infos.pop(0)
            if limits[i] is None:
                continue
            if err is not None:
                errors.append(err)
                if isinstance(getattr(err, "cause", None), Canceled):
                    canceled += 1
                else:
                    failed += 1
                continue
            nodes[i] = {"id": limits[i].node_id, "address": limits[i].address}
            hashes[i] = h
            successful += 1
            if successful >= rs.optimal_threshold():
                cancel.set()  # cancelling remaining uploads (:178-181)
        for t in threads:
            t.join()
        self.last_counts = {"total": piece_count, "optimal": rs.optimal_threshold(), "successful": successful,
                            "failed": failed, "canceled": canceled}
        joined = "; ".join(str(e) for e in errors)
        if successful <= rs.repair_threshold() and successful < rs.optimal_threshold():
            raise ECClientError(f"successful puts ({successful}) less than or equal to repair threshold "
                                f"({rs.repair_threshold()}), {joined}")
        if successful < rs.optimal_threshold():
            raise ECClientError(f"successful puts ({successful}) less than success threshold "
                                f"({rs.optimal_threshold()}), {joined}")
        return nodes, hashes

    def put_single_result(self, limits, rs, data) -> List[PieceUploadResult]:
        """PutSingleResult (client.go:77-100)."""
        nodes, hashes = self.put(limits, rs, data)
        results = [PieceUploadResult(i, nodes[i]["id"], hashes[i]) for i in range(len(nodes)) if nodes[i]]
        if len(results) < rs.optimal_threshold():
            raise ECClientError(f"uploaded results ({len(results)}) are below the optimal threshold "
                                f"({rs.optimal_threshold()})")
        return results

    # ----------------------------------------------------------- download
    def get(self, limits, es, size: int):
        """Get (client.go:269-271)."""
        return self.get_with_options(limits, es, size, error_detection=False)

    def get_with_options(self, limits: List[Optional[AddressedOrderLimit]], es, size: int,
                         error_detection: bool = False):
        """GetWithOptions (client.go:273-308): a Ranger over the `size`
        bytes of the segment, decoded from the pieces on demand."""
        if len(limits) != es.total_count():
            raise ECClientError(f"size of limits slice ({len(limits)}) does not match total count "
                                f"({es.total_count()}) of erasure scheme")
        nn = non_nil_count(limits)
        if nn < es.required_count():
            raise ECClientError(f"number of non-nil limits ({nn}) is less than required count "
                                f"({es.required_count()}) of erasure scheme")
        padded_size = calc_padded(size, es.stripe_size())
        piece_size = padded_size // es.required_count()
        rrs: Dict[int, LazyPieceRanger] = {}
        for i, lim in enumerate(limits):
            if lim is not None:
                rrs[i] = LazyPieceRanger(self.store, lim, piece_size)
        try:
            rr = streams.decode(rrs, es, self.memory_limit, error_detection or self.force_error_detection)
        except Exception as e:  # noqa: BLE001 - Error.Wrap
            raise ECClientError(str(e), e)
        return unpad(rr, padded_size - size)


class _BytesReader:
    def __init__(self, b: bytes):
        self._b, self._o = b, 0

    def read(self, n: int = -1) -> bytes:
        if n is None or n < 0:
            n = len(self._b) - self._o
        out = self._b[self._o:self._o + n]
        self._o += len(out)
        return out


class LoopbackPieceStore:
    """In-process piece store (the MockPieceStore / io.Pipe pattern of
    private/piecestore/client_test.go:76-179): put_piece stores what it reads,
    download serves byte ranges of it; `delay` (seconds per node id) and
    `fail` (node ids) model slow and bad nodes for the long-tail cut."""

    def __init__(self, delay: Optional[Dict[bytes, float]] = None, fail: Sequence[bytes] = ()):
        self.pieces: Dict[bytes, bytes] = {}
        self.delay = dict(delay or {})
        self.fail = set(fail)
        self._mu = threading.Lock()

    def put_piece(self, limit: AddressedOrderLimit, reader, cancel: threading.Event):
        if limit.node_id in self.fail:
            raise IOError("node refused the piece")
        d = self.delay.get(limit.node_id, 0.0)
        if d and cancel.wait(d):
            raise Canceled("context canceled")
        data = streams.read_all(reader)
        if cancel.is_set() and d:
            raise Canceled("context canceled")
        with self._mu:
            self.pieces[limit.node_id] = data
        return eestream_hash(data)

    def download(self, limit: AddressedOrderLimit, offset: int, length: int):
        with self._mu:
            data = self.pieces.get(limit.node_id)
        if data is None:
            return streams.fatal_read_closer(IOError("piece not found"))
        if offset + length > len(data):
            return streams.fatal_read_closer(IOError("range beyond the stored piece"))
        return _BytesReader(data[offset:offset + length])


def eestream_hash(data: bytes) -> bytes:
    """Stand-in for the PieceHash a node signs (its value is not checked here)."""
    import hashlib
    return hashlib.sha256(data).digest()
