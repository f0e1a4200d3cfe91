"""Segment-level upload integration (uplink_amd/segment.py, SURVEY §8f row
1): pieceReader.PieceReader (segmentupload/single.go:228-238) served from
one batched parity-only encode, the segment held in a pinned buffer.Backend."""
import io
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from uplink_amd import eestream, segment  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rs(k, n, ess):
    return eestream.RedundancyStrategy(eestream.RSScheme(eestream.new_fec(k, n), ess), 0, 0)


@pytest.mark.parametrize("k,n,ess,size", [(29, 80, 256, 3 * 1024 * 1024 + 123), (4, 10, 256, 1 << 20),
                                          (20, 60, 4096, 5 * 81920 - 4), (2, 4, 1024, 0),
                                          (1, 1, 64, 1000), (3, 7, 100, 5000)])
def test_piece_readers_match_oracle_and_encoded_reader(oracle, k, n, ess, size):
    rs = _rs(k, n, ess)
    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    padded = eestream.pad(data, rs.stripe_size())
    ref = oracle.FEC(k, n).encode_segment(np.frombuffer(padded, dtype=np.uint8), ess)
    spr = segment.SegmentPieceReader(data, rs)
    for num in range(n):
        piece = spr.piece_reader(num).read()
        assert len(piece) == eestream.calc_piece_size(size, rs)
        assert piece == ref[num].tobytes(), num
    for num in sorted({0, k - 1, min(k, n - 1), n - 1}):  # the reference path, per stripe
        assert eestream.new_encoded_reader(io.BytesIO(padded), rs, num).read() == ref[num].tobytes()
    spr.close()


def test_pinned_backend_as_segment_source(oracle):
    k, n, ess = 29, 80, 256
    rs = _rs(k, n, ess)
    be = segment.PinnedBackend(1 << 20)
    chunks = [os.urandom(1000), os.urandom(70000), os.urandom(123)]
    for c in chunks:
        assert be.write(c) == len(c)
    data = b"".join(chunks)
    assert be.size() == len(data)
    assert be.read_at(500, 900) == data[900:1400]
    assert be.read_at(10, len(data)) == b""
    with pytest.raises(Exception):
        be.write(b"x" * (1 << 20))
    spr = segment.SegmentPieceReader(be, rs)
    ref = oracle.FEC(k, n).encode_segment(np.frombuffer(eestream.pad(data, rs.stripe_size()), dtype=np.uint8), ess)
    for num in (0, 28, 29, 79):
        assert spr.piece_reader(num).read() == ref[num].tobytes()
    spr.close()
    be.close()
    with pytest.raises(eestream.EEStreamError):
        be.read_at(1, 0)


def test_piece_reader_num_errors():
    spr = segment.SegmentPieceReader(b"abc", _rs(4, 10, 256))
    with pytest.raises(eestream.InfectiousError, match="num must be non-negative"):
        spr.piece_reader(-1)
    with pytest.raises(eestream.InfectiousError, match="num must be less than 10"):
        spr.piece_reader(10)


@pytest.mark.parametrize("k,n,ess,stripes,nseg", [(29, 80, 256, 1000, 5), (20, 60, 4096, 300, 4), (4, 10, 256, 257, 7),
                                                  (29, 80, 256, 9040, 2)])
def test_chunked_host_pipelines(oracle, k, n, ess, stripes, nseg):
    """ec_encode_segments_host / ec_rebuild_segments_host move each segment in
    chunks of stripes over three role streams and rotate segments over three
    device slots: ragged last chunks, more segments than slots, both output
    layouts, and rebuild inputs both in one strided buffer (one 2D copy per
    chunk) and at scattered pointers (one copy per piece)."""
    import ctypes
    from uplink_amd import _native as N
    lib = N.load()
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    plen, spad = stripes * ess, stripes * k * ess
    rng = np.random.default_rng(stripes + nseg)
    segs = rng.integers(0, 256, (nseg, spad), dtype=np.uint8)
    fec = oracle.FEC(k, n)
    ref = np.stack([fec.encode_segment(segs[g], ess, threads=8) for g in range(nseg)])
    for flags, rows in ((0, n), (N.EC_FLAG_PARITY_ONLY, n - k)):
        pieces = np.zeros((nseg, rows, plen), dtype=np.uint8)
        assert lib.ec_encode_segments_host(sch.ctx, segs.ctypes.data, nseg, stripes, pieces.ctypes.data, flags) == 0
        assert np.array_equal(pieces, ref[:, n - rows:]), flags
    full = np.ascontiguousarray(ref)
    nums = sorted(rng.choice(n, k, replace=False).tolist())
    # strided: the chosen pieces inside one [nseg][n][plen] buffer
    out = np.zeros((nseg, spad), dtype=np.uint8)
    c_nums = (ctypes.c_int * k)(*nums)
    c_ptrs = (ctypes.c_void_p * k)(*[full.ctypes.data + i * plen for i in nums])
    assert lib.ec_rebuild_segments_host(sch.ctx, k, c_nums, c_ptrs, stripes, nseg, n * plen, out.ctypes.data) == 0
    assert np.array_equal(out, segs)
    # scattered: every chosen piece of every segment in its own buffer, at one segment stride
    scat = [np.ascontiguousarray(full[:, i, :]) for i in nums]  # [nseg][plen] each
    c_ptrs2 = (ctypes.c_void_p * k)(*[a.ctypes.data for a in scat[::-1]])
    c_nums2 = (ctypes.c_int * k)(*nums[::-1])
    out2 = np.zeros((nseg, spad), dtype=np.uint8)
    assert lib.ec_rebuild_segments_host(sch.ctx, k, c_nums2, c_ptrs2, stripes, nseg, plen, out2.ctypes.data) == 0
    assert np.array_equal(out2, segs)


@pytest.mark.parametrize("chunk", [0, 1, 7, 300, 100000])
def test_streamed_parity_pieces_read_in_small_reads(oracle, chunk):
    """the parity pieces arrive chunk by chunk
    (ec_upload_begin) and a piece reader waits only for the chunk holding
    the bytes it is asked for.  Pieces read in ragged small reads that cross
    chunk and stripe boundaries, interleaved over pieces, equal the oracle's;
    data pieces are gathered per read from the segment."""
    k, n, ess = 29, 80, 256
    rs = _rs(k, n, ess)
    size = 2 * 1024 * 1024 + 777
    data = np.random.default_rng(chunk + 1).integers(0, 256, size, dtype=np.uint8).tobytes()
    padded = eestream.pad(data, rs.stripe_size())
    ref = oracle.FEC(k, n).encode_segment(np.frombuffer(padded, dtype=np.uint8), ess)
    spr = segment.SegmentPieceReader(data, rs, chunk_stripes=chunk)
    readers = {num: spr.piece_reader(num) for num in (0, 5, 28, 29, 30, 54, 79)}
    got = {num: [] for num in readers}
    plen = ref.shape[1]
    rng = np.random.default_rng(3)
    left = set(readers)
    while left:
        for num in sorted(left):
            b = readers[num].read(int(rng.integers(1, 3000)))
            if not b:
                left.discard(num)
            got[num].append(b)
    for num in readers:
        assert b"".join(got[num]) == ref[num].tobytes(), num
    assert spr.ready_stripes() == plen // ess
    for r in readers.values():
        r.close()
    spr.close()
    with pytest.raises(eestream.EEStreamError):
        spr._wait(1)


def test_streamed_upload_c_abi_partial_wait_and_threads(oracle):
    """ec_upload_wait(u, s) returns once stripes [0, s) of every piece are in
    host memory -- checked right after each wait, before the upload ends --
    for the full (all n pieces) and parity-only layouts, from 8 threads
    waiting on one upload at once; argument errors."""
    import ctypes
    import threading
    from uplink_amd import _native as NAT
    lib = NAT.load()
    k, n, ess, stripes = 29, 80, 256, 3000
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    seg = np.random.default_rng(9).integers(0, 256, stripes * k * ess, dtype=np.uint8)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    assert lib.ec_upload_begin(sch.ctx, None, stripes, None, 0, 0, ctypes.byref(ctypes.c_void_p())) \
        == NAT.EC_ERR_INVALID_ARG
    assert lib.ec_upload_wait(None, 1) == NAT.EC_ERR_INVALID_ARG
    for flags, rows in ((0, n), (NAT.EC_FLAG_PARITY_ONLY, n - k)):
        pieces = segment.PinnedHost(rows * stripes * ess)
        view = pieces.array.reshape(rows, stripes * ess)
        h = ctypes.c_void_p()
        assert lib.ec_upload_begin(sch.ctx, seg.ctypes.data, stripes, pieces.ptr, flags, 0, ctypes.byref(h)) == 0
        errors = []

        def waiter(t):
            s = (t + 1) * stripes // 8
            if lib.ec_upload_wait(h, s) != 0:
                errors.append((t, "rc"))
            elif not np.array_equal(view[:, : s * ess], ref[n - rows:, : s * ess]):
                errors.append((t, s))
        th = [threading.Thread(target=waiter, args=(t,)) for t in range(8)]
        [t.start() for t in th]
        [t.join() for t in th]
        assert not errors, errors
        assert lib.ec_upload_ready(h) == stripes
        assert lib.ec_upload_end(h) == 0
        assert np.array_equal(view, ref[n - rows:])
        pieces.close()


@pytest.mark.parametrize("k,n,ess,size,chunk", [
    (29, 80, 256, 3 * 1024 * 1024 + 123, 0),    # the library's chunks (128, 256, ... 2048 stripes)
    (29, 80, 256, 2 * 1024 * 1024 + 5, 300),    # 300 stripes = 75 BLAKE3 chunks per piece chunk
    (29, 80, 256, 1024 * 1024, 7),              # 7 stripes: not whole BLAKE3 chunks -> hashed after the last
    (4, 10, 256, 1 << 20, 4),                   # 4 stripes = 1 KiB per chunk
    (20, 60, 4096, 5 * 81920 - 4, 0), (29, 80, 256, 100, 0),  # pieces of one BLAKE3 chunk: after the last
])
def test_streamed_upload_hashes_pieces(oracle, k, n, ess, size, chunk):
    """SegmentPieceReader(hash_pieces=True) streams the
    parity and hashes every piece chunk by chunk (EC_FLAG_HASH_PIECES), as the
    reference hashes each piece through a TeeReader while it streams
    (piecestore/upload.go:155,262-270).  Every piece's BLAKE3 against the
    oracle's hash of the oracle's piece -- asked before any piece is read (it
    waits only for the tree fold) -- and the piece bytes."""
    from oracle import blake3 as ob
    rs = _rs(k, n, ess)
    data = np.random.default_rng(size + chunk).integers(0, 256, size, dtype=np.uint8).tobytes()
    padded = eestream.pad(data, rs.stripe_size())
    ref = oracle.FEC(k, n).encode_segment(np.frombuffer(padded, dtype=np.uint8), ess, threads=8)
    want = ob.blake3_many(ref, threads=8)
    spr = segment.SegmentPieceReader(data, rs, hash_pieces=True, chunk_stripes=chunk)
    try:
        for num in range(n):
            assert spr.piece_hash(num) == want[num].tobytes(), num
        for num in sorted({0, k - 1, k, n - 1}):
            with _closing(spr.piece_reader(num)) as r:
                assert r.read() == ref[num].tobytes(), num
    finally:
        spr.close()


class _closing:
    def __init__(self, r):
        self.r = r

    def __enter__(self):
        return self.r

    def __exit__(self, *a):
        self.r.close()


def test_upload_hashes_c_abi(oracle):
    """ec_upload_begin(EC_FLAG_HASH_PIECES): all n hashes for the full layout
    and the parity-only one; ec_upload_hashes on an upload begun without the
    flag is an argument error; unknown flags are refused."""
    import ctypes
    from oracle import blake3 as ob
    from uplink_amd import _native as NAT
    lib = NAT.load()
    k, n, ess, stripes = 29, 80, 256, 2100
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    seg = np.random.default_rng(21).integers(0, 256, stripes * k * ess, dtype=np.uint8)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    want = ob.blake3_many(ref, threads=8)
    assert lib.ec_upload_begin(sch.ctx, seg.ctypes.data, stripes, seg.ctypes.data, 0x80, 0,
                               ctypes.byref(ctypes.c_void_p())) == NAT.EC_ERR_INVALID_ARG
    for flags, rows in ((NAT.EC_FLAG_HASH_PIECES, n), (NAT.EC_FLAG_HASH_PIECES | NAT.EC_FLAG_PARITY_ONLY, n - k),
                        (NAT.EC_FLAG_PARITY_ONLY, n - k)):
        pieces = segment.PinnedHost(rows * stripes * ess)
        h = ctypes.c_void_p()
        assert lib.ec_upload_begin(sch.ctx, seg.ctypes.data, stripes, pieces.ptr, flags, 0, ctypes.byref(h)) == 0
        hashes = np.zeros((n, 32), dtype=np.uint8)
        rc = lib.ec_upload_hashes(h, hashes.ctypes.data)
        if flags & NAT.EC_FLAG_HASH_PIECES:
            assert rc == 0 and np.array_equal(hashes, want), flags
        else:
            assert rc == NAT.EC_ERR_INVALID_ARG
        assert lib.ec_upload_end(h) == 0
        assert np.array_equal(pieces.array.reshape(rows, -1), ref[n - rows:])
        pieces.close()


def test_piece_stream_keeps_buffers_after_reader_close(oracle):
    """a piece stream still being read keeps the reader's
    pinned buffers; closing (or dropping) the reader hands them back to the
    pool only after its last stream closes.  Another segment's reader, taking
    buffers of the same size from the pool meanwhile, must not change what the
    first reader's open streams return."""
    import gc
    k, n, ess = 29, 80, 256
    rs = _rs(k, n, ess)
    size = 1024 * 1024
    rng = np.random.default_rng(31)
    d1, d2 = (rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(2))
    ref1 = oracle.FEC(k, n).encode_segment(np.frombuffer(eestream.pad(d1, rs.stripe_size()), dtype=np.uint8), ess)
    a = segment.SegmentPieceReader(d1, rs)
    data_stream, parity_stream = a.piece_reader(3), a.piece_reader(40)
    first = data_stream.read(1000)
    a.close()  # streams open: the buffers stay with them
    with pytest.raises(eestream.EEStreamError):
        a.piece_reader(4)
    b = segment.SegmentPieceReader(d2, rs)  # same sizes: would take the pool's buffers
    assert len(b.piece_reader(40).read()) > 0 and len(b.piece_reader(3).read()) > 0
    assert first + data_stream.read() == ref1[3].tobytes()
    assert parity_stream.read() == ref1[40].tobytes()
    data_stream.close()
    parity_stream.close()  # the last one: a's buffers go back now
    b.close()
    # dropping a reader whose streams are alive: the streams hold it, nothing is released under them
    c = segment.SegmentPieceReader(d1, rs)
    s3 = c.piece_reader(3)
    del c
    gc.collect()
    d = segment.SegmentPieceReader(d2, rs)
    d.piece_reader(3).read()
    assert s3.read() == ref1[3].tobytes()
    s3.close()
    d.close()


def test_upload_end_waits_for_callers_inside():
    """ec_upload_end while other threads are inside
    ec_upload_wait / _ready on the same handle returns only after they have
    left (no use of the freed handle)."""
    import ctypes
    import threading
    import time
    from uplink_amd import _native as NAT
    lib = NAT.load()
    k, n, ess, stripes = 29, 80, 256, 9040
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    seg = segment.PinnedHost(stripes * k * ess)
    seg.array[:] = 7
    pieces = segment.PinnedHost((n - k) * stripes * ess)
    for rep in range(3):
        h = ctypes.c_void_p()
        assert lib.ec_upload_begin(sch.ctx, seg.ptr, stripes, pieces.ptr, NAT.EC_FLAG_PARITY_ONLY, 0,
                                   ctypes.byref(h)) == 0
        go = threading.Barrier(9)
        rcs = []

        def waiter(t):
            go.wait()
            rcs.append(lib.ec_upload_wait(h, stripes) if t % 2 else int(lib.ec_upload_ready(h) >= 0))
        th = [threading.Thread(target=waiter, args=(t,)) for t in range(8)]
        [t.start() for t in th]
        go.wait()
        time.sleep(0.02)  # the waiters are inside their calls
        assert lib.ec_upload_end(h) == 0
        [t.join() for t in th]
        assert all(r in (0, 1, NAT.EC_ERR_INVALID_ARG) for r in rcs), rcs
    seg.close()
    pieces.close()


def test_reader_used_after_close_allocates_nothing():
    """piece_reader / piece_hash after close() raise before
    any buffer is taken from the pool or any upload is begun (the buffers went
    back to the pool at close; a new upload would be reclaimed only by
    __del__)."""
    rs = _rs(29, 80, 256)
    data = np.random.default_rng(5).integers(0, 256, 100000, dtype=np.uint8).tobytes()
    for touch_first in (False, True):
        spr = segment.SegmentPieceReader(data, rs, hash_pieces=True)
        if touch_first:
            spr.piece_reader(30).read()
        spr.close()
        for call in (lambda: spr.piece_reader(1), lambda: spr.piece_reader(40), lambda: spr.piece_hash(2)):
            with pytest.raises(eestream.EEStreamError, match="after close"):
                call()
            assert spr._upload is None and spr._bufs == [] and spr._padded is None
