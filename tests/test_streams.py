"""The eestream stream layer (uplink_amd/streams.py) against the reference's
own stream tests (private/eestream/rs_test.go): EncodeReader2 ->
DecodeReaders2 round trips, the fault-injection tables of testRSProblematic
(errors, EOF, early EOF, late EOF, random data with error detection, slow
readers), stalled readers, the Decode / EncodedRanger rangers, and the
batched ReadStripes.

Every test runs twice: with the engine (RSScheme over the GPU C-ABI, marked
gpu) and with a test-only scheme backed by the CPU oracle, which exercises
the same host logic on a machine without a GPU."""
import io
import os
import time

import numpy as np
import pytest

from uplink_amd import eestream, streams

HERE = os.path.dirname(os.path.abspath(__file__))


class OracleScheme:
    """ErasureScheme + the batch methods streams.py calls, computed by the
    CPU oracle (storj.io/infectious restatement).  Test infrastructure."""

    def __init__(self, oracle, k, n, ess):
        self.fec = oracle.FEC(k, n)
        self.O = oracle
        self.k, self.n, self.ess = k, n, ess
        self.rebuild_calls = 0

    def required_count(self):
        return self.k

    def total_count(self):
        return self.n

    def erasure_share_size(self):
        return self.ess

    def stripe_size(self):
        return self.k * self.ess

    def _map(self, e):
        if getattr(e, "code", None) == -10:
            return eestream.NotEnoughShares(str(e))
        if getattr(e, "code", None) == -13:
            return eestream.TooManyErrors(str(e))
        return eestream.InfectiousError(str(e))

    def encode_stripes(self, data):
        return self.fec.encode_segment(np.asarray(data, dtype=np.uint8), self.ess)

    def rebuild_stripes(self, nums, pieces, nstripes):
        self.rebuild_calls += 1
        try:
            return self.fec.rebuild_segment(list(nums), [np.asarray(p) for p in pieces], self.ess)
        except self.O.OracleError as e:
            raise self._map(e)

    def decode(self, out, shares):
        try:
            return self.fec.decode([s.number for s in shares], [s.data for s in shares])
        except self.O.OracleError as e:
            raise self._map(e)


class CountingScheme:
    """Wraps the GPU scheme to count batched rebuild calls."""

    def __init__(self, inner):
        self.inner = inner
        self.rebuild_calls = 0

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def rebuild_stripes(self, nums, pieces, nstripes):
        self.rebuild_calls += 1
        return self.inner.rebuild_stripes(nums, pieces, nstripes)


@pytest.fixture(params=["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def make_rs(request, oracle):
    if request.param == "gpu":
        torch = pytest.importorskip("torch")
        if not torch.cuda.is_available():
            pytest.skip("no GPU")

        def mk(k, n, ess, repair=0, optimal=0):
            return eestream.RedundancyStrategy(CountingScheme(eestream.RSScheme(eestream.new_fec(k, n), ess)),
                                               repair, optimal)
    else:
        def mk(k, n, ess, repair=0, optimal=0):
            return eestream.RedundancyStrategy(OracleScheme(oracle, k, n, ess), repair, optimal)
    return mk


def _read_all_pieces(readers):
    out = [streams.read_all(r) for r in readers]
    for r in readers:
        r.close()
    return out


def _byte_reader(b):
    return streams.nop_closer(io.BytesIO(b))


def test_rs(make_rs):
    """TestRS (rs_test.go:32-60)."""
    data = os.urandom(32 * 1024)
    rs = make_rs(2, 4, 8 * 1024)
    readers = streams.encode_reader2(io.BytesIO(data), rs)
    dec = streams.decode_readers2(dict(enumerate(readers)), rs, 32 * 1024, 0, False)
    try:
        assert streams.read_all(dec) == data
    finally:
        assert dec.close() is None


def test_rs_unexpected_eof(make_rs):
    """TestRSUnexpectedEOF (rs_test.go:64-91): ReadFull past the end."""
    data = os.urandom(32 * 1024)
    rs = make_rs(2, 4, 8 * 1024)
    readers = streams.encode_reader2(io.BytesIO(data), rs)
    dec = streams.decode_readers2(dict(enumerate(readers)), rs, 32 * 1024, 0, False)
    with pytest.raises(EOFError, match="unexpected EOF"):
        streams.read_full(dec, len(data) + 1024)
    dec.close()


def test_rs_ranger(make_rs):
    """TestRSRanger (rs_test.go:93-153) without its AES-GCM transform (out of
    scope): PadReader -> EncodeReader2 -> ByteRangers ->
    Decode -> UnpadSlow, plus unaligned sub-ranges of the decoded ranger."""
    data = os.urandom(32 * 1024)
    rs = make_rs(2, 4, 8 * 1024)
    padded = eestream.pad(data, 2 * rs.stripe_size())
    pieces = _read_all_pieces(streams.encode_reader2(io.BytesIO(padded), rs))
    rrs = {i: streams.ByteRanger(p) for i, p in enumerate(pieces)}
    rr = streams.decode(rrs, rs, 0, False)
    assert rr.size() == len(padded)
    got = streams.read_all(rr.range(0, rr.size()))
    assert eestream.unpad(got) == data
    rng = np.random.default_rng(5)
    for _ in range(4):
        off = int(rng.integers(0, len(padded) - 1))
        ln = int(rng.integers(0, len(padded) - off))
        assert streams.read_all(rr.range(off, ln)) == padded[off:off + ln]


def test_decode_ranger_errors(make_rs):
    rs = make_rs(2, 4, 1024)
    with pytest.raises(eestream.EEStreamError, match="not enough readers to reconstruct data!"):
        streams.decode({0: streams.ByteRanger(b"x" * 1024)}, rs)
    with pytest.raises(eestream.EEStreamError, match="range reader sizes don't all match"):
        streams.decode({0: streams.ByteRanger(b"x" * 1024), 1: streams.ByteRanger(b"x" * 2048)}, rs)
    with pytest.raises(eestream.EEStreamError, match=r"range reader size \(1000\) must be a multiple"):
        streams.decode({0: streams.ByteRanger(b"x" * 1000), 1: streams.ByteRanger(b"x" * 1000)}, rs)
    with pytest.raises(eestream.EEStreamError, match="negative max buffer memory"):
        streams.decode({}, rs, -1)
    r = streams.decode_readers2({}, rs, -1)
    with pytest.raises(eestream.EEStreamError, match="negative expected size"):
        r.read(1)
    r = streams.decode_readers2({}, rs, 1000)
    with pytest.raises(eestream.EEStreamError, match=r"expected size \(1000\) not a factor decoded block size \(2048\)"):
        r.read(1)


def test_encoded_ranger(make_rs, oracle):
    """EncodedRanger (encode.go:213-268): OutputSize and unaligned ranges
    equal the matching bytes of every piece."""
    k, n, ess = 3, 7, 512
    rs = make_rs(k, n, ess)
    data = os.urandom(9 * k * ess)
    er = streams.new_encoded_ranger(streams.ByteRanger(data), rs)
    assert er.output_size() == 9 * ess
    full = oracle.FEC(k, n).encode_segment(np.frombuffer(data, dtype=np.uint8), ess)
    for off, ln in [(0, 9 * ess), (100, 1000), (ess, 2 * ess), (7 * ess + 3, 2 * ess - 3)]:
        outs = er.range(off, ln)
        assert len(outs) == n
        for i, r in enumerate(outs):
            assert streams.read_all(r) == full[i, off:off + ln].tobytes()
    with pytest.raises(eestream.EEStreamError, match="must be a multiple of erasure encoder block size"):
        streams.new_encoded_ranger(streams.ByteRanger(b"x" * 100), rs)


def test_encode_reader2_partial_stripe(make_rs):
    """A stream that does not end on a stripe boundary: io.ReadFull's
    unexpected EOF in every piece (encode.go:180)."""
    rs = make_rs(2, 4, 1024)
    readers = streams.encode_reader2(io.BytesIO(os.urandom(2048 * 3 + 100)), rs)
    with pytest.raises(EOFError, match="unexpected EOF"):
        streams.read_all(readers[0])


# ------------------------------------------------------------------ testRSProblematic
def _problematic(rs_factory, tt, fn):
    size, ess, k, n, problematic, fail, detect = tt
    data = os.urandom(size)
    rs = rs_factory(k, n, ess)
    pieces = _read_all_pieces(streams.encode_reader2(io.BytesIO(data), rs))
    rmap = {}
    for i in range(problematic):
        rmap[i] = fn(pieces[i])
    for i in range(problematic, n):
        rmap[i] = _byte_reader(pieces[i])
    dec = streams.decode_readers2(rmap, rs, size, 3 * 1024, detect)
    try:
        try:
            got, err = streams.read_all(dec), None
        except Exception as e:  # noqa: BLE001 - the reference checks err != nil
            got, err = None, e
        if fail:
            assert err is not None or got != data, f"expected to fail: {tt}"
        else:
            assert err is None, f"{tt}: {err}"
            assert got == data
    finally:
        assert dec.close() is None


def _table(rows, detect):
    return [(s, b, k, n, p, f, detect) for (s, b, k, n, p, f) in rows]


K4, K6 = 4 * 1024, 6 * 1024
ERR_TABLE = [(K4, 1024, 1, 1, 0, False), (K4, 1024, 1, 1, 1, True), (K4, 1024, 1, 2, 0, False),
             (K4, 1024, 1, 2, 1, False), (K4, 1024, 1, 2, 2, True), (K4, 1024, 2, 4, 0, False),
             (K4, 1024, 2, 4, 1, False), (K4, 1024, 2, 4, 2, False), (K4, 1024, 2, 4, 3, True),
             (K4, 1024, 2, 4, 4, True), (K6, 1024, 3, 7, 0, False), (K6, 1024, 3, 7, 1, False),
             (K6, 1024, 3, 7, 2, False), (K6, 1024, 3, 7, 3, False), (K6, 1024, 3, 7, 4, False),
             (K6, 1024, 3, 7, 5, True), (K6, 1024, 3, 7, 6, True), (K6, 1024, 3, 7, 7, True)]


@pytest.mark.parametrize("tt", _table(ERR_TABLE, False))
def test_rs_errors(make_rs, tt):
    """TestRSErrors (rs_test.go:194-221): FatalReadCloser pieces."""
    _problematic(make_rs, tt, lambda p: streams.fatal_read_closer(RuntimeError("I am an error piece")))


@pytest.mark.parametrize("tt", _table(ERR_TABLE, False))
def test_rs_eof(make_rs, tt):
    """TestRSEOF (rs_test.go:224-251): EOF at byte 0."""
    _problematic(make_rs, tt, lambda p: streams.limit_read_closer(_byte_reader(p), 0))


@pytest.mark.parametrize("tt", _table(ERR_TABLE, False))
def test_rs_early_eof(make_rs, tt):
    """TestRSEarlyEOF (rs_test.go:254-282): EOF after 500 bytes."""
    _problematic(make_rs, tt, lambda p: streams.limit_read_closer(_byte_reader(p), 500))


@pytest.mark.parametrize("tt", _table([r[:5] + (False,) for r in ERR_TABLE], False))
def test_rs_late_eof(make_rs, tt):
    """TestRSLateEOF (rs_test.go:285-314): random trailing bytes."""
    rng = np.random.default_rng(tt[4])
    _problematic(make_rs, tt, lambda p: _byte_reader(p + os.urandom(1 + int(rng.integers(0, 10000)))))


RANDOM_TABLE = [(K4, 1024, 1, 1, 0, False), (K4, 1024, 1, 1, 1, True), (K4, 1024, 1, 2, 0, False),
                (K4, 1024, 1, 2, 1, True), (K4, 1024, 1, 2, 2, True), (K4, 1024, 2, 4, 0, False),
                (K4, 1024, 2, 4, 1, False), (K4, 1024, 2, 4, 2, True), (K4, 1024, 2, 4, 3, True),
                (K4, 1024, 2, 4, 4, True), (K6, 1024, 3, 7, 0, False), (K6, 1024, 3, 7, 1, False),
                (K6, 1024, 3, 7, 2, False), (K6, 1024, 3, 7, 4, True), (K6, 1024, 3, 7, 5, True),
                (K6, 1024, 3, 7, 6, True), (K6, 1024, 3, 7, 7, True)]


@pytest.mark.parametrize("tt", _table(RANDOM_TABLE, True))
def test_rs_random_data(make_rs, tt):
    """TestRSRandomData (rs_test.go:317-342): random bytes in place of the
    first pieces, error detection on (Berlekamp-Welch)."""
    _problematic(make_rs, tt, lambda p: _byte_reader(os.urandom(len(p))))


class _Slow:
    def __init__(self, b, delay):
        self._r, self._d = io.BytesIO(b), delay

    def read(self, n=-1):
        time.sleep(self._d)
        return self._r.read(n)

    def close(self):
        return None


SLOW_TABLE = [(K4, 1024, 1, 1, 0, False), (K4, 1024, 1, 2, 0, False), (K4, 1024, 2, 4, 0, False),
              (K4, 1024, 2, 4, 1, False), (K6, 1024, 3, 7, 0, False), (K6, 1024, 3, 7, 1, False),
              (K6, 1024, 3, 7, 2, False), (K6, 1024, 3, 7, 3, False)]


@pytest.mark.parametrize("tt", _table(SLOW_TABLE, False))
def test_rs_slow(make_rs, tt):
    """TestRSSlow (rs_test.go:345-364): 1 s per read must not be waited for."""
    start = time.monotonic()
    _problematic(make_rs, tt, lambda p: _Slow(p, 1.0))
    assert time.monotonic() - start < 1.0, "waited for slow reader"


def test_encoder_stalled_readers(make_rs):
    """TestEncoderStalledReaders (rs_test.go:457-483): 25 of 60 piece
    readers never read; the rest finish without waiting for them."""
    rs = make_rs(30, 60, 1024, 35, 50)
    readers = streams.encode_reader2(io.BytesIO(os.urandom(120 * 1024)), rs)
    start = time.monotonic()
    for r in readers[25:]:
        assert len(streams.read_all(r)) == 4 * 1024
    assert time.monotonic() - start < 1.0
    for r in readers:
        assert r.close() is None


def test_decoder_error_with_stalled_readers(make_rs):
    """TestDecoderErrorWithStalledReaders (rs_test.go:503-544): 4 good, 3
    slow, 13 failing readers for k = 10: the error comes without waiting."""
    rs = make_rs(10, 20, 1024)
    pieces = _read_all_pieces(streams.encode_reader2(io.BytesIO(os.urandom(10 * 1024)), rs))
    rmap = {i: _byte_reader(pieces[i]) for i in range(4)}
    rmap.update({i: _Slow(pieces[i], 1.0) for i in range(4, 7)})
    rmap.update({i: streams.fatal_read_closer(RuntimeError("I am an error piece")) for i in range(7, 20)})
    dec = streams.decode_readers2(rmap, rs, 10 * 1024, 0, False)
    start = time.monotonic()
    with pytest.raises(eestream.EEStreamError, match="error retrieving piece 07: I am an error piece"):
        streams.read_all(dec)
    assert time.monotonic() - start < 1.0, "waited for slow reader"
    dec.close()


def test_read_stripes_batches(make_rs):
    """§8f row 2: with a large ReadStripes buffer the whole run of ready
    stripes is rebuilt by one batched call (one share choice / inversion),
    here RS(29,80), ess 256, 300 stripes, decoded from 29 parity pieces."""
    k, n, ess, stripes = 29, 80, 256, 300
    rs = make_rs(k, n, ess)
    data = os.urandom(stripes * k * ess)
    pieces = _read_all_pieces(streams.encode_reader2(io.BytesIO(data), rs))
    rmap = {i: _byte_reader(pieces[i]) for i in range(n - k, n)}
    dec = streams.decode_readers2(rmap, rs, len(data), 0, False, out_buffer=len(data))
    assert streams.read_all(dec) == data
    dec.close()
    assert 1 <= rs.scheme.rebuild_calls <= 3  # one per ReadStripes (readers race the core)
    # the reference's 32 KiB buffer: at most 4 stripes per call
    rs.scheme.rebuild_calls = 0
    rmap = {i: _byte_reader(pieces[i]) for i in range(n - k, n)}
    dec = streams.decode_readers2(rmap, rs, len(data), 0, False)
    assert streams.read_all(dec) == data
    dec.close()
    assert rs.scheme.rebuild_calls >= stripes // (32 * 1024 // (k * ess))


def test_read_stripes_unexpected_next_stripe(make_rs):
    rs = make_rs(2, 4, 1024)
    pieces = _read_all_pieces(streams.encode_reader2(io.BytesIO(os.urandom(4096)), rs))
    sr = streams.new_stripe_reader({i: _byte_reader(p) for i, p in enumerate(pieces)}, rs, 2, False)
    with pytest.raises(eestream.EEStreamError, match="unexpected next stripe"):
        sr.read_stripes(1)
    data, count = sr.read_stripes(0)
    assert count >= 1 and len(data) == count * 2048
    sr.close()


def test_error_detection_runs(make_rs):
    """forceErrorDetection over long runs (§8f row 3): RS(29,80), 64
    stripes, 36 pieces offered of which 3 return random bytes; every run of
    stripes is corrected by one Decode (Berlekamp-Welch, e = 3)."""
    k, n, ess, stripes = 29, 80, 256, 64
    rs = make_rs(k, n, ess)
    data = os.urandom(stripes * k * ess)
    pieces = _read_all_pieces(streams.encode_reader2(io.BytesIO(data), rs))
    nums = sorted(np.random.default_rng(11).choice(n, 36, replace=False).tolist())
    bad = set(nums[::12])  # 3 corrupted pieces
    rmap = {i: _byte_reader(os.urandom(len(pieces[i])) if i in bad else pieces[i]) for i in nums}
    dec = streams.decode_readers2(rmap, rs, len(data), 0, True, out_buffer=len(data))
    assert streams.read_all(dec) == data
    dec.close()
