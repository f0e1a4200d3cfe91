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
