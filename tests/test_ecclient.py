"""The ecclient mirror (uplink_amd/ecclient.py): the
upload fan-out of put / PutSingleResult (private/ecclient/client.go:77-209)
and the download sizing of GetWithOptions (client.go:273-308, 333-339),
against the reference's own test (client_test.go:16-46, TestUnique), its
pinned error texts, and round trips through a loopback piece store -- on the
CPU with the oracle-backed test scheme, and on the GPU with the engine,
including the production 67,254,016-byte encrypted segment (9060 stripes up,
9059 down: SURVEY Appendix B)."""
import io
import os

import numpy as np
import pytest

from test_streams import OracleScheme
from uplink_amd import ecclient, eestream, streams

HERE = os.path.dirname(os.path.abspath(__file__))


def limits_for(n, seed=0):
    rng = np.random.default_rng(seed)
    return [ecclient.AddressedOrderLimit(node_id=bytes(rng.integers(1, 256, 32, dtype=np.uint8)), address=f"n{i}")
            for i in range(n)]


@pytest.mark.parametrize("size,block,want", [
    (0, 7424, 0), (1, 7424, 7424), (7424, 7424, 7424), (7425, 7424, 14848),
    (64 << 20, 7424, 9040 * 7424),            # synthetic 64 MiB segment: 9040 stripes
    (67_254_016, 7424, 67_254_016),           # production encrypted segment: 9059 stripes exactly
])
def test_calc_padded(size, block, want):
    assert ecclient.calc_padded(size, block) == want


def test_unique_like_reference():
    """TestUnique (client_test.go:16-46)."""
    lim = limits_for(4)
    cases = [
        (None, True), ([], True), ([lim[0]], True), ([lim[0], lim[1]], True), ([lim[0], lim[0]], False),
        ([lim[0], lim[1], lim[0]], False), ([lim[1], lim[0], lim[0]], False), ([lim[0], lim[0], lim[1]], False),
        ([lim[2], lim[0], lim[1]], True), ([lim[2], lim[0], lim[3], lim[1]], True),
        ([lim[2], lim[0], lim[2], lim[1]], False), ([lim[1], lim[0], lim[3], lim[1]], False),
    ]
    for i, (ls, want) in enumerate(cases):
        assert ecclient.unique(ls) == want, f"case {i}"
    assert ecclient.unique([lim[0], None, None, lim[1]])  # nil limits are not duplicates


@pytest.fixture
def cpu_rs(oracle):
    return eestream.RedundancyStrategy(OracleScheme(oracle, 4, 10, 256), repair_threshold=6, optimal_threshold=8)


def test_put_argument_errors(cpu_rs):
    c = ecclient.ECClient(ecclient.LoopbackPieceStore())
    lim = limits_for(10)
    with pytest.raises(ecclient.ECClientError, match=r"^ecclient: size of limits slice \(9\) does not match total "
                                                     r"count \(10\) of erasure scheme$"):
        c.put(lim[:9], cpu_rs, io.BytesIO(b"x"))
    with pytest.raises(ecclient.ECClientError, match=r"number of non-nil limits \(5\) is less than or equal to the "
                                                     r"repair threshold \(6\) of erasure scheme"):
        c.put(lim[:5] + [None] * 5, cpu_rs, io.BytesIO(b"x"))
    with pytest.raises(ecclient.ECClientError, match="duplicated nodes are not allowed"):
        c.put([lim[0]] + lim[:9], cpu_rs, io.BytesIO(b"x"))


def test_get_argument_errors(cpu_rs):
    c = ecclient.ECClient(ecclient.LoopbackPieceStore())
    lim = limits_for(10)
    with pytest.raises(ecclient.ECClientError, match=r"size of limits slice \(11\) does not match total count \(10\)"):
        c.get_with_options(lim + lim[:1], cpu_rs, 100)
    with pytest.raises(ecclient.ECClientError, match=r"number of non-nil limits \(3\) is less than required count "
                                                     r"\(4\) of erasure scheme"):
        c.get_with_options(lim[:3] + [None] * 7, cpu_rs, 100)


def _roundtrip(rs, size, seed, slow=(), bad=(), missing_on_download=()):
    rng = np.random.default_rng(seed)
    data = rng.bytes(size)
    lim = limits_for(rs.total_count(), seed)
    store = ecclient.LoopbackPieceStore(delay={lim[i].node_id: 2.0 for i in slow},
                                        fail=[lim[i].node_id for i in bad])
    c = ecclient.ECClient(store)
    nodes, hashes = c.put(lim, rs, io.BytesIO(data))
    stored = [i for i in range(len(lim)) if nodes[i]]
    assert len(stored) >= rs.optimal_threshold()
    assert not set(stored) & set(bad)
    # the download offers only the pieces that were stored, minus some
    dl = [lim[i] if (nodes[i] and i not in missing_on_download) else None for i in range(len(lim))]
    rr = c.get_with_options(dl, rs, size)
    assert rr.size() == size
    got = streams.read_all(rr.range(0, size))
    assert got == data
    # a ranged read inside the segment (block-aligned internally, like decodedRanger)
    if size > 3000:
        assert streams.read_all(rr.range(1234, 1700)) == data[1234:1234 + 1700]
    return c, store, lim, nodes


def test_put_get_roundtrip_cpu(cpu_rs):
    """RS(4,10), optimal 8: slow nodes are cut by the long-tail cancel once 8
    pieces are stored (client.go:178-181), a bad node fails; the download
    decodes from the remaining pieces, sized by calcPadded and Unpad
    (sizes just below a stripe multiple: the upload has one stripe more)."""
    c, store, lim, nodes = _roundtrip(cpu_rs, 1 << 20, 1, slow=(3, 7), missing_on_download=(0, 1))
    assert c.last_counts["canceled"] == 2 and c.last_counts["failed"] == 0
    assert nodes[3] is None and nodes[7] is None
    c, store, lim, nodes = _roundtrip(cpu_rs, 7424 * 3 - 2, 2, slow=(9,), bad=(5,), missing_on_download=(2,))
    assert c.last_counts["canceled"] == 1 and c.last_counts["failed"] == 1
    assert nodes[9] is None and nodes[5] is None


class _BrokenOnCancelStore(ecclient.LoopbackPieceStore):
    """Slow nodes that fail with a plain I/O error (not context.Canceled) once
    the long-tail cut has canceled them, as a transport torn down under them
    does."""

    def put_piece(self, limit, reader, cancel):
        if limit.node_id in self.delay:
            cancel.wait(self.delay[limit.node_id])
            if cancel.is_set():
                raise IOError("connection reset by peer")
        return super().put_piece(limit, reader, cancel)


def test_put_error_after_cut_counts_as_canceled(cpu_rs):
    """client.go:232-243: once the pieces context is canceled, PutPiece
    reports the upload as cut due to a slow connection (context.Canceled the
    primary error) whatever the store returned; a failure before the cut stays
    an "upload failed"."""
    rng = np.random.default_rng(11)
    lim = limits_for(10, 11)
    store = _BrokenOnCancelStore(delay={lim[2].node_id: 5.0, lim[6].node_id: 5.0})
    c = ecclient.ECClient(store)
    nodes, _ = c.put(lim, cpu_rs, io.BytesIO(rng.bytes(50_000)))
    assert c.last_counts == {"total": 10, "optimal": 8, "successful": 8, "failed": 0, "canceled": 2}
    assert nodes[2] is None and nodes[6] is None


def test_put_canceled_by_user(cpu_rs):
    """client.go:232-243 tells a user cancel (the parent context)
    from the long-tail cut: with the caller's context canceled while uploads
    are in flight, every upload still running fails as "upload canceled by
    user" with context.Canceled first in the chain, and put fails below the
    repair threshold."""
    import threading
    rng = np.random.default_rng(12)
    lim = limits_for(10, 12)
    store = _BrokenOnCancelStore(delay={l.node_id: 5.0 for l in lim})
    c = ecclient.ECClient(store)
    parent = threading.Event()
    threading.Timer(0.2, parent.set).start()
    with pytest.raises(ecclient.ECClientError) as ei:
        c.put(lim, cpu_rs, io.BytesIO(rng.bytes(20_000)), parent=parent)
    msg = str(ei.value)
    assert "successful puts (0) less than or equal to repair threshold" in msg
    assert "upload canceled by user: connection reset by peer" in msg and "slow connection" not in msg
    assert c.last_counts["canceled"] == 10 and c.last_counts["failed"] == 0


def test_put_single_result_cpu(cpu_rs):
    c = ecclient.ECClient(ecclient.LoopbackPieceStore())
    res = c.put_single_result(limits_for(10, 3), cpu_rs, io.BytesIO(b"hello" * 999))
    assert len(res) >= 8 and len({r.piece_num for r in res}) == len(res)
    assert all(r.node_id and r.hash for r in res)


def test_put_below_thresholds_cpu(cpu_rs):
    lim = limits_for(10, 4)
    store = ecclient.LoopbackPieceStore(fail=[lim[i].node_id for i in range(5)])
    with pytest.raises(ecclient.ECClientError, match=r"successful puts \(5\) less than or equal to repair threshold "
                                                     r"\(6\), .*node refused the piece"):
        ecclient.ECClient(store).put(lim, cpu_rs, io.BytesIO(b"y" * 5000))
    store = ecclient.LoopbackPieceStore(fail=[lim[i].node_id for i in range(3)])
    with pytest.raises(ecclient.ECClientError, match=r"successful puts \(7\) less than success threshold \(8\)"):
        ecclient.ECClient(store).put(lim, cpu_rs, io.BytesIO(b"y" * 5000))


@pytest.mark.gpu
def test_production_segment_up_and_down_on_gpu():
    """RS(29,80) with production thresholds (repair 35, optimal 65), ess 256,
    the 67,254,016-byte encrypted 64 MiB segment: the upload pads to 9060
    stripes (2,319,360-byte pieces), GetWithOptions reads 9059 stripes
    (2,319,104-byte piece ranges) and Unpad(0) -- the engine does both
    codings; 15 slow nodes are cut by the long tail, and the download uses 40
    of the 65 stored pieces."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rs = eestream.RedundancyStrategy(eestream.RSScheme(eestream.new_fec(29, 80), 256), 35, 65)
    size = 67_254_016
    slow = tuple(range(50, 65))
    c, store, lim, nodes = _roundtrip(rs, size, 29, slow=slow, missing_on_download=tuple(range(0, 25)))
    lens = {len(v) for v in store.pieces.values()}
    assert lens == {2_319_360}
    assert ecclient.calc_padded(size, rs.stripe_size()) // 29 == 2_319_104
    assert c.last_counts["successful"] == 65 and c.last_counts["canceled"] == 15
