"""GPU parity: the HIP kernels behind include/uplink_ec.h against the oracle
(CPU restatement of storj.io/infectious) and the golden fixtures.  Bit-exact
is the only bar (byte-field arithmetic).  Mirrors the reference's test
strategy: round trips over many (k, n, ess), fault tables,
piece sizes, error strings, plus full-size BASELINE configurations."""
import ctypes
import json
import os
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from uplink_amd import _native, eestream  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def scheme(k, n, ess):
    return eestream.RSScheme(eestream.new_fec(k, n), ess)


def gpu_encode(sch, seg: np.ndarray, nseg=1, parity_only=False):
    k, n, ess = sch.fc.k, sch.fc.n, sch.ess
    stripes = seg.size // (nseg * k * ess)
    d_seg = torch.from_numpy(seg).cuda()
    rows = n - k if parity_only else n
    d_pieces = torch.full((nseg, rows, stripes * ess), 0xAB, dtype=torch.uint8, device="cuda")
    eestream.SegmentCodec(sch).encode_segments(d_seg, nseg, stripes, d_pieces, parity_only=parity_only)
    torch.cuda.synchronize()
    return d_pieces


def gpu_rebuild(sch, d_pieces, nums, stripes, nseg=1):
    k, n, ess = sch.fc.k, sch.fc.n, sch.ess
    plen = stripes * ess
    rows = d_pieces.shape[1]
    base = d_pieces.data_ptr()
    out = torch.full((nseg, stripes * k * ess), 0xCD, dtype=torch.uint8, device="cuda")
    eestream.SegmentCodec(sch).rebuild_segments(nums, [base + i * plen for i in nums], stripes, out, nseg=nseg,
                                                piece_seg_stride=rows * plen, out_seg_stride=stripes * k * ess)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def prepare_code(sch, nums):
    """Have the share set's straight-line code made now (the batched rebuild
    otherwise makes it in the background after the set's first launch)."""
    arr = (ctypes.c_int * len(nums))(*nums)
    return sch._lib.ec_prepare_rebuild(sch._ctx, len(nums), arr, 1)


def test_golden_fixtures_on_gpu():
    with open(os.path.join(HERE, "golden", "manifest.json")) as fh:
        man = json.load(fh)
    for case in man["cases"]:
        z = np.load(os.path.join(HERE, "golden", case["file"]))
        k, n, ess, stripes = case["k"], case["n"], case["ess"], case["stripes"]
        sch = scheme(k, n, ess)
        assert np.array_equal(sch.generator(), z["generator"])
        d_pieces = gpu_encode(sch, z["segment"])
        assert np.array_equal(d_pieces.cpu().numpy()[0], z["pieces"]), case["file"]
        for nums in (list(range(n - k, n)), sorted(np.random.default_rng(7).choice(n, k, replace=False).tolist())):
            assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], z["segment"])


CONFIGS = [  # (k, n, ess, stripes): reference test configs + BASELINE shapes + edge cases
    (1, 1, 64, 5), (1, 2, 64, 3), (2, 4, 1024, 3), (3, 7, 1024, 4), (4, 10, 256, 1025), (10, 20, 1024, 10),
    (20, 60, 4096, 3), (29, 80, 256, 100), (30, 60, 1024, 7), (50, 80, 256, 3), (20, 50, 8192, 2),
    (2, 4, 8, 5),        # ess < 16: byte kernel
    (3, 5, 100, 4),      # ess not a multiple of 16: byte kernel
    (7, 200, 256, 2),    # 193 parity rows: split over launches
    (29, 80, 256, 1),    # a single stripe (tile tail)
    (29, 80, 256, 129),  # ragged tile count
    (64, 96, 256, 17),   # k > 48: runtime-matrix encoder (no run-time compilation)
    (128, 256, 256, 3),  # the limits: 128 inputs, 128 parity rows (4 passes of 32), all-parity rebuild of 128 rows
]


@pytest.mark.parametrize("k,n,ess,stripes", CONFIGS)
def test_encode_rebuild_vs_oracle(oracle, k, n, ess, stripes):
    rng = np.random.default_rng(k * 1000 + n + ess)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=4)
    d_pieces = gpu_encode(sch, seg)
    got = d_pieces.cpu().numpy()[0]
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert len(bad) == 0, f"pieces differ: {bad[:8]}"
    sets = [list(range(n - k, n)), sorted(rng.choice(n, k, replace=False).tolist()), list(range(k))]
    for nums in sets:
        assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg), nums


def test_full_size_rs_29_80_64mib(oracle):
    """BASELINE configs[1]/[2]: RS(29,80), 64 MiB segment (PadReader-padded to
    9040 stripes), encode bit-exact vs the oracle, decode from exactly 29."""
    k, n, ess = 29, 80, 256
    raw = np.random.default_rng(0x5EED0000).integers(0, 256, 64 * 2**20, dtype=np.uint8)
    seg = oracle.pad(raw, k * ess)
    assert seg.size == 9040 * k * ess
    sch = scheme(k, n, ess)
    d_pieces = gpu_encode(sch, seg)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=min(os.cpu_count() or 1, 16))
    assert np.array_equal(d_pieces.cpu().numpy()[0], ref)
    for body in (_native.EC_BODY_AUTO, _native.EC_BODY_JUMP_TABLE):
        assert sch._lib.ec_set_body(sch._ctx, body) == 0
        for nums in (list(range(51, 80)), sorted(np.random.default_rng(29).choice(80, 29, replace=False).tolist())):
            # EC_BODY_AUTO: a share set's first launch on the jump table (the share-set pass), the
            # next ones on generated code once it is made (here: waited for)
            for use in range(2 if body == _native.EC_BODY_AUTO else 1):
                if use == 1:
                    assert prepare_code(sch, nums) == 1
                out = gpu_rebuild(sch, d_pieces, nums, 9040)[0]
                assert np.array_equal(out, seg)
                assert eestream.unpad(out.tobytes()) == raw.tobytes()
                want = _native.EC_BODY_JUMP_TABLE if body == _native.EC_BODY_JUMP_TABLE or use == 0 else \
                    _native.EC_BODY_STRAIGHT_LINE
                assert sch._lib.ec_last_body(sch._ctx) == want


def test_full_size_rs_20_60_ess4096(oracle):
    """BASELINE configs[4] shape: RS(20,60), 4 KiB shares, 64 MiB segment."""
    k, n, ess = 20, 60, 4096
    raw = np.random.default_rng(5).integers(0, 256, 64 * 2**20, dtype=np.uint8)
    seg = oracle.pad(raw, k * ess)
    sch = scheme(k, n, ess)
    d_pieces = gpu_encode(sch, seg)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=min(os.cpu_count() or 1, 16))
    assert np.array_equal(d_pieces.cpu().numpy()[0], ref)
    out = gpu_rebuild(sch, d_pieces, list(range(40, 60)), seg.size // (k * ess))[0]
    assert np.array_equal(out, seg)


def test_batched_segments_and_parity_only(oracle):
    k, n, ess, stripes, nseg = 29, 80, 256, 37, 3
    rng = np.random.default_rng(11)
    segs = rng.integers(0, 256, nseg * stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    d_pieces = gpu_encode(sch, segs, nseg=nseg)
    d_par = gpu_encode(sch, segs, nseg=nseg, parity_only=True)
    f = oracle.FEC(k, n)
    for g in range(nseg):
        ref = f.encode_segment(segs[g * stripes * k * ess:(g + 1) * stripes * k * ess], ess)
        assert np.array_equal(d_pieces[g].cpu().numpy(), ref)
        assert np.array_equal(d_par[g].cpu().numpy(), ref[k:])
    nums = sorted(rng.choice(n, k, replace=False).tolist())
    out = gpu_rebuild(sch, d_pieces, nums, stripes, nseg=nseg)
    assert np.array_equal(out.reshape(-1), segs)


def test_rebuild_share_choice_and_errors():
    """infectious Rebuild semantics through the C-ABI: unsorted and > k shares,
    data pass-through, NotEnoughShares, invalid share id."""
    k, n, ess, stripes = 3, 7, 256, 5
    seg = np.random.default_rng(2).integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    d_pieces = gpu_encode(sch, seg)
    assert np.array_equal(gpu_rebuild(sch, d_pieces, [6, 2, 0, 4, 5], stripes)[0], seg)
    with pytest.raises(eestream.NotEnoughShares):
        gpu_rebuild(sch, d_pieces, [0, 1], stripes)
    with pytest.raises(eestream.InfectiousError, match="invalid share id"):
        gpu_rebuild(sch, d_pieces[:, :], [0, 1, 7], stripes)


def test_unaligned_buffers_take_byte_path(oracle):
    k, n, ess, stripes = 4, 10, 256, 9
    seg = np.random.default_rng(3).integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    buf = torch.zeros(seg.size + 1, dtype=torch.uint8, device="cuda")
    buf[1:] = torch.from_numpy(seg).cuda()
    pieces = torch.zeros(n * stripes * ess + 3, dtype=torch.uint8, device="cuda")
    lib = _native.load()
    rc = lib.ec_encode_segments(sch.ctx, buf.data_ptr() + 1, 1, stripes, pieces.data_ptr() + 3, 0,
                                torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    got = pieces.cpu().numpy()[3:].reshape(n, -1)
    assert np.array_equal(got, oracle.FEC(k, n).encode_segment(seg, ess))


# ------------------------------------------------------------ scheme surface
def test_encode_single_and_encode_match_oracle(oracle):
    for k, n, ess in [(2, 4, 8 * 1024), (29, 80, 256), (3, 7, 100), (1, 4, 64)]:
        sch = scheme(k, n, ess)
        f = oracle.FEC(k, n)
        stripe = np.random.default_rng(k).integers(0, 256, k * ess, dtype=np.uint8)
        out = np.zeros(ess, dtype=np.uint8)
        for num in range(n):
            sch.encode_single(stripe, out, num)
            assert np.array_equal(out, f.encode_single(stripe, num)), (k, n, num)
        got = {}
        sch.encode(stripe, lambda num, data: got.__setitem__(num, data.copy()))
        ref = f.encode(stripe)
        assert sorted(got) == list(range(n))
        for num in range(n):
            assert np.array_equal(got[num], ref[num])


def test_encode_single_error_strings():
    # segmentupload/encode_test.go:53,63 with RS(required 1, total 4), ess 64
    rs = eestream.new_redundancy_strategy_from_storj(1, 2, 3, 4, 64)
    data = np.ones(rs.stripe_size(), dtype=np.uint8)
    out = np.zeros(64, dtype=np.uint8)
    with pytest.raises(eestream.InfectiousError) as e1:
        rs.encode_single(data, out, -1)
    assert str(e1.value) == "num must be non-negative"
    with pytest.raises(eestream.InfectiousError) as e2:
        rs.encode_single(data, out, rs.total_count())
    assert str(e2.value) == "num must be less than 4"


def test_encoded_reader():
    """TestEncodedReader (segmentupload/encode_test.go:16-68)."""
    import io
    rs = eestream.new_redundancy_strategy_from_storj(1, 2, 3, 4, 64)
    expected = bytes([1]) * rs.stripe_size()
    pieces = []
    for i in range(rs.total_count()):
        r = eestream.new_encoded_reader(io.BytesIO(expected), rs, i)
        pieces.append(eestream.Share(i, np.frombuffer(r.read(), dtype=np.uint8)))
    assert rs.decode(None, pieces).tobytes() == expected
    r = eestream.new_encoded_reader(io.BytesIO(bytes([1]) * (rs.stripe_size() - 1)), rs, 0)
    for _ in range(2):
        with pytest.raises(EOFError, match="unexpected EOF"):
            r.read()
    for num, msg in [(-1, "num must be non-negative"), (rs.total_count(), "num must be less than 4")]:
        r = eestream.new_encoded_reader(io.BytesIO(bytes([1]) * rs.stripe_size()), rs, num)
        for _ in range(2):
            with pytest.raises(eestream.InfectiousError) as ei:
                r.read()
            assert str(ei.value) == msg


def _encode_pieces(rs, data: bytes):
    import io
    return [np.frombuffer(eestream.new_encoded_reader(io.BytesIO(data), rs, i).read(), dtype=np.uint8)
            for i in range(rs.total_count())]


def _decode_stream(rs, pieces: dict, nstripes: int, error_detection: bool):
    """Stripe-by-stripe decode the way StripeReader.ReadStripes drives the
    scheme (stripe.go:382-428): Rebuild, or Decode with error detection."""
    ess, k = rs.erasure_share_size(), rs.required_count()
    out = bytearray()
    for s in range(nstripes):
        shares = [eestream.Share(num, np.array(p[s * ess:(s + 1) * ess])) for num, p in sorted(pieces.items())]
        if error_detection:
            out += rs.decode(None, shares).tobytes()
        else:
            buf = bytearray(k * ess)

            def put(sh):
                buf[sh.number * ess:(sh.number + 1) * ess] = sh.data.tobytes()
            rs.rebuild(shares, put)
            out += buf
    return bytes(out)


def test_rs_roundtrip_like_testrs():
    """TestRS (rs_test.go:32-60): RS(2,4), ess 8 KiB, 32 KiB."""
    rs = eestream.RedundancyStrategy(scheme(2, 4, 8 * 1024), 0, 0)
    data = os.urandom(32 * 1024)
    pieces = _encode_pieces(rs, data)
    assert _decode_stream(rs, dict(enumerate(pieces)), 2, False) == data


# the fault tables of rs_test.go:194-342 at the scheme level: pieces that
# error / EOF are missing; random-data pieces are corrupt (error detection)
FAULT_TABLE = [  # (dataSize, blockSize, required, total, problematic)
    (4 * 1024, 1024, 1, 1, 0), (4 * 1024, 1024, 1, 2, 0), (4 * 1024, 1024, 1, 2, 1), (4 * 1024, 1024, 2, 4, 0),
    (4 * 1024, 1024, 2, 4, 1), (4 * 1024, 1024, 2, 4, 2), (6 * 1024, 1024, 3, 7, 0), (6 * 1024, 1024, 3, 7, 1),
    (6 * 1024, 1024, 3, 7, 2), (6 * 1024, 1024, 3, 7, 3), (6 * 1024, 1024, 3, 7, 4),
    (4 * 1024, 1024, 1, 1, 1), (4 * 1024, 1024, 1, 2, 2), (4 * 1024, 1024, 2, 4, 3), (6 * 1024, 1024, 3, 7, 5),
]


@pytest.mark.parametrize("size,ess,k,n,problematic", FAULT_TABLE)
def test_missing_pieces_table(size, ess, k, n, problematic):
    """TestRSErrors / TestRSEOF: the first `problematic` pieces are
    unavailable; decoding works iff at least k remain."""
    rs = eestream.RedundancyStrategy(scheme(k, n, ess), 0, 0)
    data = os.urandom(size)
    pieces = _encode_pieces(rs, data)
    avail = {i: pieces[i] for i in range(problematic, n)}
    nstripes = size // (k * ess)
    if len(avail) < k:
        with pytest.raises(eestream.NotEnoughShares):
            _decode_stream(rs, avail, nstripes, False)
    else:
        assert _decode_stream(rs, avail, nstripes, False) == data


@pytest.mark.parametrize("size,ess,k,n,problematic,fail", [
    # TestRSRandomData (rs_test.go:317-342) with errorDetection=true and all pieces offered
    (4 * 1024, 1024, 2, 4, 0, False), (4 * 1024, 1024, 2, 4, 1, False), (4 * 1024, 1024, 2, 4, 2, True),
    (6 * 1024, 1024, 3, 7, 0, False), (6 * 1024, 1024, 3, 7, 1, False), (6 * 1024, 1024, 3, 7, 2, False),
    (6 * 1024, 1024, 3, 7, 4, True), (4 * 1024, 1024, 1, 2, 1, True),
])
def test_random_data_pieces_error_detection(size, ess, k, n, problematic, fail):
    rs = eestream.RedundancyStrategy(scheme(k, n, ess), 0, 0)
    data = os.urandom(size)
    pieces = _encode_pieces(rs, data)
    rng = np.random.default_rng(problematic)
    avail = {i: (rng.integers(0, 256, len(pieces[i]), dtype=np.uint8) if i < problematic else pieces[i])
             for i in range(n)}
    nstripes = size // (k * ess)
    if fail:
        try:
            got = _decode_stream(rs, avail, nstripes, True)
        except (eestream.NotEnoughShares, eestream.TooManyErrors):
            return
        assert got != data
    else:
        assert _decode_stream(rs, avail, nstripes, True) == data


def test_decode_corrects_scattered_errors_rs_29_80(oracle):
    k, n, ess = 29, 80, 256
    sch = scheme(k, n, ess)
    rng = np.random.default_rng(8)
    stripe = rng.integers(0, 256, k * ess, dtype=np.uint8)
    allsh = oracle.FEC(k, n).encode(stripe)
    nums = sorted(rng.choice(n, 45, replace=False).tolist())  # e = 8
    shares = [eestream.Share(i, np.array(allsh[i])) for i in nums]
    for i in rng.choice(45, 8, replace=False):
        shares[i].data[rng.integers(0, ess, 20)] ^= rng.integers(1, 256, 20, dtype=np.uint8)
    got = sch.decode(None, shares)
    assert np.array_equal(got, stripe)
    # Decode corrects the shares in place (infectious semantics)
    for s in shares:
        assert np.array_equal(s.data, allsh[s.number])


def test_calc_piece_size_matches_encoded_reader():
    rs = eestream.RedundancyStrategy(scheme(2, 4, 1024), 0, 0)
    import io
    for size in (0, 1, 1020, 1024, 32764, 32768, 32868):
        padded = eestream.pad(os.urandom(size), rs.stripe_size())
        for i in range(rs.total_count()):
            piece = eestream.new_encoded_reader(io.BytesIO(padded), rs, i).read()
            assert len(piece) == eestream.calc_piece_size(size, rs)


def test_concurrent_encode_single(oracle):
    """EncodeSingle is called from many goroutines at once (uplink.go:83)."""
    k, n, ess = 29, 80, 256
    sch = scheme(k, n, ess)
    f = oracle.FEC(k, n)
    rng = np.random.default_rng(12)
    stripes = [rng.integers(0, 256, k * ess, dtype=np.uint8) for _ in range(6)]
    errors = []

    def work(t):
        out = np.zeros(ess, dtype=np.uint8)
        for rep in range(10):
            s = stripes[(t + rep) % len(stripes)]
            num = (t * 7 + rep * 13) % n
            sch.encode_single(s, out, num)
            if not np.array_equal(out, f.encode_single(s, num)):
                errors.append((t, rep))
    th = [threading.Thread(target=work, args=(t,)) for t in range(12)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors


def test_coalesced_encode_single_mixed_sizes(oracle):
    """ec_encode_single coalesces concurrent calls into batched launches
    (group commit, grouped by share size): 48 threads with share sizes 256
    (compile-time encoder), 64 and 100 (byte kernel), data and parity rows,
    every result against the oracle."""
    k, n = 29, 80
    sch = scheme(k, n, 256)
    f = oracle.FEC(k, n)
    rng = np.random.default_rng(13)
    sizes = (256, 64, 100)
    stripes = {bs: [rng.integers(0, 256, k * bs, dtype=np.uint8) for _ in range(4)] for bs in sizes}
    errors = []

    def work(t):
        bs = sizes[t % len(sizes)]
        out = np.zeros(bs, dtype=np.uint8)
        for rep in range(25):
            s = stripes[bs][(t + rep) % 4]
            num = (t * 11 + rep * 17) % n
            sch.encode_single(s, out, num)
            if not np.array_equal(out, f.encode_single(s, num)):
                errors.append((t, rep, bs, num))
    th = [threading.Thread(target=work, args=(t,)) for t in range(48)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]


def test_concurrent_rebuild_and_decode_more_threads_than_workspaces(oracle):
    """40 threads of per-stripe Rebuild and Decode on one context -- more
    callers than its 8 workspaces, so most of them wait and are handed a
    workspace in arrival order -- with random share sets and, for Decode, one
    corrupted share; every result against the stripe it came from."""
    k, n, ess = 29, 80, 256
    sch = scheme(k, n, ess)
    f = oracle.FEC(k, n)
    rng = np.random.default_rng(17)
    stripes = [rng.integers(0, 256, k * ess, dtype=np.uint8) for _ in range(6)]
    allsh = [f.encode(s) for s in stripes]
    errors = []

    def work(t):
        r = np.random.default_rng(1000 + t)
        for rep in range(10):
            i = (t + rep) % len(stripes)
            if t % 2 == 0:
                nums = sorted(r.choice(n, k, replace=False).tolist())
                got = np.zeros(k * ess, dtype=np.uint8)

                def put(sh, got=got):
                    got[sh.number * ess:(sh.number + 1) * ess] = sh.data
                sch.rebuild([eestream.Share(j, np.array(allsh[i][j])) for j in nums], put)
            else:
                nums = sorted(r.choice(n, k + 4, replace=False).tolist())
                sh = [eestream.Share(j, np.array(allsh[i][j])) for j in nums]
                sh[int(r.integers(0, len(sh)))].data[int(r.integers(0, ess))] ^= 0x5A
                got = sch.decode(None, sh)
            if not np.array_equal(np.asarray(got).reshape(-1), stripes[i]):
                errors.append((t, rep))
    th = [threading.Thread(target=work, args=(t,)) for t in range(40)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]


def _pinned(lib, nbytes):
    p = lib.ec_host_alloc(nbytes)
    assert p
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    return p, arr


def test_host_pipeline_encode_rebuild(oracle):
    """ec_encode_segments_host / ec_rebuild_segments_host: pinned host
    buffers in and out, 3-stream H2D/kernel/D2H ring (end-to-end path)."""
    lib = _native.load()
    k, n, ess, stripes, nseg = 20, 60, 4096, 9, 5
    sch = scheme(k, n, ess)
    spad, plen = stripes * k * ess, stripes * ess
    ps, segs = _pinned(lib, nseg * spad)
    segs[:] = np.random.default_rng(31).integers(0, 256, nseg * spad, dtype=np.uint8)
    pp, pieces = _pinned(lib, nseg * n * plen)
    po, out = _pinned(lib, nseg * spad)
    try:
        assert lib.ec_encode_segments_host(sch.ctx, ps, nseg, stripes, pp, 0) == 0
        f = oracle.FEC(k, n)
        for g in range(nseg):
            ref = f.encode_segment(segs[g * spad:(g + 1) * spad], ess)
            assert np.array_equal(pieces[g * n * plen:(g + 1) * n * plen].reshape(n, plen), ref)
        nums = list(range(40, 60))
        c_nums = (ctypes.c_int * k)(*nums)
        c_ptrs = (ctypes.c_void_p * k)(*[pp + i * plen for i in nums])
        assert lib.ec_rebuild_segments_host(sch.ctx, k, c_nums, c_ptrs, stripes, nseg, n * plen, po) == 0
        assert np.array_equal(out, segs)
    finally:
        for p in (ps, pp, po):
            lib.ec_host_free(p)


def test_c1_loopback_piecestore(oracle):
    """BASELINE configs[0] / SURVEY §8d C1: RS(4,10), ess 256, a 1 MiB
    segment through the upload path (PadReader, one EncodedReader per piece,
    segmentupload/encode.go:16-75) into an in-process piece store (the
    MockPieceStore role, piecestore/client_test.go:136-179), then downloaded
    from pieces {6,7,8,9} and from a seeded random 4-subset (Rebuild over all
    stripes, stripe.go:382-428) and unpadded."""
    import io
    k, n, ess = 4, 10, 256
    rs = eestream.RedundancyStrategy(scheme(k, n, ess), 0, 0)
    data = np.random.default_rng(20261015).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    padded = eestream.pad(data, rs.stripe_size())
    stripes = len(padded) // rs.stripe_size()
    assert stripes == 1025
    store = {}
    for num in range(n):
        piece = eestream.new_encoded_reader(io.BytesIO(padded), rs, num).read()
        assert len(piece) == eestream.calc_piece_size(len(data), rs)
        store[num] = piece
    ref = oracle.FEC(k, n).encode_segment(np.frombuffer(padded, dtype=np.uint8), ess)
    for num in range(n):
        assert np.array_equal(np.frombuffer(store[num], dtype=np.uint8), ref[num])
    d_pieces = torch.from_numpy(np.stack([np.frombuffer(store[i], dtype=np.uint8) for i in range(n)])).cuda()
    d_pieces = d_pieces.reshape(1, n, -1)
    rng = np.random.default_rng(4)
    for nums in ([6, 7, 8, 9], sorted(rng.choice(n, k, replace=False).tolist())):
        out = gpu_rebuild(rs.scheme, d_pieces, nums, stripes)[0]
        assert eestream.unpad(out.tobytes()) == data


def test_unsafe_rs_scheme_decode_is_rebuild(oracle):
    """NewUnsafeRSScheme (unsafe_rs.go:32-52): Decode = Rebuild into out,
    no correction -- a corrupted share among the chosen k shows through,
    where RSScheme.Decode corrects it."""
    k, n, ess = 4, 10, 512
    fc = eestream.new_fec(k, n)
    safe, unsafe = eestream.RSScheme(fc, ess), eestream.new_unsafe_rs_scheme(fc, ess)
    stripe = np.random.default_rng(21).integers(0, 256, k * ess, dtype=np.uint8)
    allsh = oracle.FEC(k, n).encode(stripe)
    shares = [eestream.Share(i, np.array(allsh[i])) for i in (9, 7, 5, 3)]
    out = np.zeros(k * ess + 7, dtype=np.uint8)
    got = unsafe.decode(out, shares)
    assert np.array_equal(got, stripe) and got.base is out or np.shares_memory(got, out)
    bad = [eestream.Share(i, np.array(allsh[i])) for i in (0, 2, 4, 6, 8, 9)]
    bad[1].data[3] ^= 0x41  # share 2: one of the shares Rebuild takes
    assert not np.array_equal(unsafe.decode(None, [s.deep_copy() for s in bad]), stripe)
    assert np.array_equal(safe.decode(None, bad), stripe)


BODIES = [pytest.param(_native.EC_BODY_JUMP_TABLE, id="jt"), pytest.param(_native.EC_BODY_STRAIGHT_LINE, id="sl")]


@pytest.mark.parametrize("body", BODIES)
@pytest.mark.parametrize("k,n", [(29, 80), (20, 60), (50, 80)])
def test_rebuild_every_missing_count(oracle, k, n, body):
    """Rebuild with every number m of missing data shares, 0..min(k, n-k):
    this walks every rebuild kernel width (2, 3 or 4 waves of up to 8 rows,
    several passes beyond 32 rows), every right-aligned entry point into the
    call sequence, and the copy-only case m = 0 -- through the jump table and
    through each plan's generated straight-line code."""
    ess, stripes = 256, 40
    sch = scheme(k, n, ess)
    assert sch._lib.ec_set_body(sch._ctx, body) == 0
    rng = np.random.default_rng(k * 1000 + n)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    d_pieces = gpu_encode(sch, seg)
    for m in range(0, min(k, n - k) + 1):
        data = sorted(rng.choice(k, k - m, replace=False).tolist())
        parity = sorted(rng.choice(np.arange(k, n), m, replace=False).tolist())
        nums = data + parity
        assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg), m
        if m > 0:
            assert sch._lib.ec_last_body(sch._ctx) == body


@pytest.mark.parametrize("depth", [0, 2, 3])
def test_rebuild_prefetch_depths_bit_exact(oracle, monkeypatch, depth):
    """The rebuild's input pipeline (rs_matmul_dma: LDS-DMA of the next
    chunk(s) of input shares, counted vmcnt waits, in-place slicing) at every
    prefetch depth the library builds, and the register-staged kernel (depth
    0), straight-line and jump-table bodies, against the segment: every missing count of RS(29,80) and
    RS(50,80) (2-4 waves), a 2-segment batch with a ragged last tile, and an
    RS(128,256) parity-heavy set (8 waves, two passes).  The depth is set at
    ec_create and is library-wide, so the test ends by creating a context at
    the default depth again."""
    monkeypatch.setenv("UPLINK_EC_REBUILD_DEPTH", str(depth))
    try:
        for k, n, stripes, nseg, body in [(29, 80, 41, 2, _native.EC_BODY_STRAIGHT_LINE),
                                          (29, 80, 41, 2, _native.EC_BODY_JUMP_TABLE),
                                          (50, 80, 9, 1, _native.EC_BODY_STRAIGHT_LINE)]:
            sch = scheme(k, n, 256)
            assert sch._lib.ec_set_body(sch._ctx, body) == 0
            rng = np.random.default_rng(depth * 100 + k)
            seg = rng.integers(0, 256, nseg * stripes * k * 256, dtype=np.uint8)
            d_pieces = gpu_encode(sch, seg, nseg=nseg)
            for m in range(0, min(k, n - k) + 1):
                nums = sorted(rng.choice(k, k - m, replace=False).tolist()) + \
                    sorted(rng.choice(np.arange(k, n), m, replace=False).tolist())
                got = gpu_rebuild(sch, d_pieces, nums, stripes, nseg=nseg)
                assert np.array_equal(got.reshape(-1), seg), (k, m)
        k, n, stripes = 128, 256, 3
        sch = scheme(k, n, 256)
        assert sch._lib.ec_set_body(sch._ctx, _native.EC_BODY_STRAIGHT_LINE) == 0
        rng = np.random.default_rng(depth)
        seg = rng.integers(0, 256, stripes * k * 256, dtype=np.uint8)
        ref = oracle.FEC(k, n).encode_segment(seg, 256, threads=4)
        d_pieces = torch.from_numpy(np.ascontiguousarray(ref)).cuda().reshape(1, n, -1)
        nums = sorted(rng.choice(np.arange(k, n), 100, replace=False).tolist()) + list(range(28))
        assert np.array_equal(gpu_rebuild(sch, d_pieces, sorted(nums), stripes)[0], seg)
        assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_STRAIGHT_LINE
    finally:
        monkeypatch.delenv("UPLINK_EC_REBUILD_DEPTH")
        scheme(29, 80, 256)  # back to the default depth


@pytest.mark.parametrize("k,n,ess,stripes", [c for c in CONFIGS if c[2] % 16 == 0])
def test_straight_line_body_vs_oracle(oracle, k, n, ess, stripes):
    """Every bit-sliced configuration with the straight-line body forced:
    rebuilds from three share sets, and the encode of the (k, n) without a
    compile-time encoder (RS(64,96), RS(128,256): their parity plans, up to 128
    rows, run as generated code too), bit-exact against the oracle."""
    rng = np.random.default_rng(k * 7 + n + ess)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    assert sch._lib.ec_set_body(sch._ctx, _native.EC_BODY_STRAIGHT_LINE) == 0
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=4)
    assert np.array_equal(gpu_encode(sch, seg).cpu().numpy()[0], ref)
    d_pieces = torch.from_numpy(np.ascontiguousarray(ref)).cuda().reshape(1, n, -1)
    for nums in (list(range(n - k, n)), sorted(rng.choice(n, k, replace=False).tolist())):
        assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg), nums
        if any(x >= k for x in nums):  # RS(128,256)'s plans take the 2-MiB code region
            assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_STRAIGHT_LINE


def test_auto_body_uses_straight_line_for_segments(oracle):
    """EC_BODY_AUTO: a whole segment's rebuild runs the plan's generated code
    from the plan's second launch on (the first, which may be its only one,
    runs the jump table: no code generation or module load for a share set
    seen once), a per-stripe call the jump table; all bit-exact."""
    k, n, ess, stripes = 29, 80, 256, 600  # 75 tiles of 2048 columns (the threshold is 64)
    rng = np.random.default_rng(77)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    d_pieces = gpu_encode(sch, seg)
    nums = list(range(n - k, n))
    assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg)
    assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_JUMP_TABLE
    assert prepare_code(sch, nums) == 1  # (queued by the first launch, made in the background)
    assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg)
    assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_STRAIGHT_LINE
    assert np.array_equal(gpu_rebuild(sch, d_pieces[:, :, :ess].contiguous(), nums, 1)[0], seg[:k * ess])
    assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_JUMP_TABLE
    assert sch._lib.ec_set_body(sch._ctx, 3) == _native.EC_ERR_INVALID_ARG


LIBRARY_ENCODERS = {(29, 80), (20, 60), (4, 10), (2, 4), (20, 50), (30, 60), (50, 80)}  # rs_encoder_aot.def


@pytest.mark.parametrize("seed", range(12))
def test_random_codes_both_bodies(oracle, seed):
    """Randomised: a random (k, n), share size and stripe count (some launches
    above the 64-tile threshold, some below), a random share set with a random
    number of extra shares, rebuilt through both bodies and the default, each
    bit-exact against the oracle's encode of the same segment."""
    rng = np.random.default_rng(seed * 7919 + 1)
    k = int(rng.integers(1, 65))
    n = int(rng.integers(k + 1, min(k + 70, 257)))
    ess = int(rng.choice([16, 64, 256, 512, 4096]))
    stripes = int(rng.integers(1, 2 + (1 << 22) // (k * ess)))
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    d_pieces = torch.from_numpy(np.ascontiguousarray(ref)).cuda().reshape(1, n, -1)
    nums = sorted(rng.choice(n, k + int(rng.integers(0, n - k + 1)), replace=False).tolist())
    # an encode that could start a run-time compilation (k <= 48, no library-built encoder) runs only
    # on generated code here: a compilation nobody waits for would hold the process at exit
    jit_able = ess % 16 == 0 and k <= 48 and n - k <= 96 and (k, n) not in LIBRARY_ENCODERS
    for body in (_native.EC_BODY_JUMP_TABLE, _native.EC_BODY_STRAIGHT_LINE, _native.EC_BODY_AUTO):
        assert sch._lib.ec_set_body(sch._ctx, body) == 0
        if body == _native.EC_BODY_STRAIGHT_LINE or not jit_able:
            assert np.array_equal(gpu_encode(sch, seg).cpu().numpy()[0], ref), (k, n, ess, stripes, body)
        assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg), (k, n, ess, stripes, body, nums)


def test_per_stripe_calls_on_generated_code_many_threads(oracle):
    """24 threads of per-stripe Rebuild and Decode with the straight-line body
    forced: most calls make a new plan and module (random share sets, more
    than the 64 cached plans, so plans are evicted and their modules unloaded
    while other threads launch), every result against the stripe."""
    k, n, ess = 20, 40, 256
    sch = scheme(k, n, ess)
    assert sch._lib.ec_set_body(sch._ctx, _native.EC_BODY_STRAIGHT_LINE) == 0
    f = oracle.FEC(k, n)
    rng = np.random.default_rng(23)
    stripes = [rng.integers(0, 256, k * ess, dtype=np.uint8) for _ in range(4)]
    allsh = [f.encode(st) for st in stripes]
    errors = []

    def work(t):
        r = np.random.default_rng(500 + t)
        try:
            for rep in range(8):
                i = (t + rep) % len(stripes)
                if rep % 2 == 0:
                    nums = sorted(r.choice(n, k, replace=False).tolist())
                    got = np.zeros(k * ess, dtype=np.uint8)

                    def put(sh, got=got):
                        got[sh.number * ess:(sh.number + 1) * ess] = sh.data
                    sch.rebuild([eestream.Share(j, np.array(allsh[i][j])) for j in nums], put)
                else:
                    nums = sorted(r.choice(n, k + 2, replace=False).tolist())
                    sh = [eestream.Share(j, np.array(allsh[i][j])) for j in nums]
                    sh[int(r.integers(0, len(sh)))].data[int(r.integers(0, ess))] ^= 0x77
                    got = sch.decode(None, sh)
                if not np.array_equal(np.asarray(got).reshape(-1), stripes[i]):
                    errors.append((t, rep))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))
    th = [threading.Thread(target=work, args=(t,)) for t in range(24)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]
    assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_STRAIGHT_LINE


def test_straight_line_plans_evicted_and_shared_across_threads(oracle):
    """Straight-line plan lifecycle: 70 share sets (past the 64 cached plans,
    so evicted plans unload their modules) rebuild whole segments on
    generated code, then 8 threads rebuild concurrently on the same new
    share sets, racing to make each plan's module once; every result
    against the segment."""
    k, n, ess, stripes = 4, 10, 256, 512  # 64 tiles per segment
    sch = scheme(k, n, ess)
    assert sch._lib.ec_set_body(sch._ctx, _native.EC_BODY_STRAIGHT_LINE) == 0  # generated code from the first launch
    rng = np.random.default_rng(91)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    d_pieces = gpu_encode(sch, seg)
    import itertools
    sets = [list(c) for c in itertools.combinations(range(n), k) if any(x >= k for x in c)]
    rng.shuffle(sets)
    for nums in sets[:70]:
        assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg), nums
        assert sch._lib.ec_last_body(sch._ctx) == _native.EC_BODY_STRAIGHT_LINE
    errors = []
    fresh = sets[70:74]

    def work(t):
        try:
            for rep in range(6):
                nums = fresh[(t + rep) % len(fresh)]
                out = torch.empty(stripes * k * ess, dtype=torch.uint8, device="cuda")
                st = torch.cuda.Stream()
                with torch.cuda.stream(st):
                    eestream.SegmentCodec(sch).rebuild_segments(
                        nums, [d_pieces.data_ptr() + j * stripes * ess for j in nums], stripes, out, nseg=1,
                        piece_seg_stride=n * stripes * ess, out_seg_stride=stripes * k * ess)
                st.synchronize()
                if not np.array_equal(out.cpu().numpy(), seg):
                    errors.append((t, rep))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))
    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]


@pytest.mark.parametrize("body", BODIES)
@pytest.mark.parametrize("extra,bad,scatter", [(2, 1, 0), (4, 1, 0), (4, 2, 0), (6, 2, 40), (8, 3, 200), (4, 3, 0)])
def test_decode_bad_pieces_over_long_runs(oracle, extra, bad, scatter, body):
    """Decode (Correct + Rebuild) of shares covering many stripes, with whole
    shares corrupted (bad pieces: every column flagged) plus scattered errors
    in one other share.  ec_decode locates the bad shares on a sample of
    columns, rewrites them from the others, and sends only the columns the
    others disagree on to per-column Berlekamp-Welch; the result must be the
    codeword, the shares corrected in place, and TooManyErrors beyond e."""
    k, n, ln = 29, 80, 4096
    sch = scheme(k, n, 256)
    assert sch._lib.ec_set_body(sch._ctx, body) == 0  # the re-encode and rebuild plans on either body
    rng = np.random.default_rng(extra * 100 + bad * 10 + scatter)
    data = rng.integers(0, 256, k * ln, dtype=np.uint8)
    allsh = oracle.FEC(k, n).encode(data)  # [n][ln]: byte column c of every share is one codeword
    nums = sorted(rng.choice(n, k + extra, replace=False).tolist())
    recv = [np.array(allsh[i]) for i in nums]
    bad_idx = [int(i) for i in rng.choice(k + extra, bad, replace=False)]
    for i in bad_idx:
        recv[i] ^= rng.integers(1, 256, ln, dtype=np.uint8)
    if scatter:
        j = [i for i in range(k + extra) if i not in bad_idx][0]
        where = rng.choice(ln, scatter, replace=False)
        recv[j][where] ^= rng.integers(1, 256, scatter, dtype=np.uint8)
    shares = [eestream.Share(nu, r.copy()) for nu, r in zip(nums, recv)]
    if bad + (1 if scatter else 0) > extra // 2:
        with pytest.raises(eestream.InfectiousError):
            sch.decode(None, shares)
        return
    assert np.array_equal(sch.decode(None, shares), data)
    for s in shares:  # corrected in place (infectious semantics)
        assert np.array_equal(s.data, allsh[s.number])
    # the same inputs through the oracle's per-column decode
    assert np.array_equal(oracle.FEC(k, n).decode(nums, [r.copy() for r in recv]), data)


# ---- compile-time-G encoders for any (k, n) (rs_encoder.hpp) ----------------

def _kernel_name(sch):
    return sch._lib.ec_encode_kernel_name(sch._ctx).decode()


@pytest.mark.parametrize("k,n", [(20, 50), (30, 60), (50, 80), (2, 4)])
def test_reference_bench_configs_use_library_encoders(oracle, k, n):
    """BenchmarkReedSolomonErasureScheme's configurations
    (private/eestream/rs_test.go:553-634) are built into the library: 8 MiB of
    stripes, all pieces and parity only, bit-exact vs the oracle.  RS(50,80)
    stages its 50 inputs in two chunks (rs_encoder.hpp kMaxChunk)."""
    ess = 256
    stripes = (8 << 20) // (k * ess)
    sch = scheme(k, n, ess)
    rng = np.random.default_rng(k * 131 + n)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    # default: at most 32 parity rows run on the parity plan's straight-line code; with the
    # jump-table body selected, on the library-built compile-time encoder
    for body, name in ((_native.EC_BODY_AUTO, "straight-line"), (_native.EC_BODY_JUMP_TABLE, "special")):
        assert sch._lib.ec_set_body(sch._ctx, body) == 0
        assert _kernel_name(sch) == name
        assert np.array_equal(gpu_encode(sch, seg).cpu().numpy()[0], ref)
        assert np.array_equal(gpu_encode(sch, seg, parity_only=True).cpu().numpy()[0], ref[k:])


@pytest.mark.parametrize("k,n,stripes", [(5, 9, 33), (37, 50, 17), (10, 20, 1025), (3, 70, 40), (36, 40, 9),
                                          (2, 98, 7)])
def test_run_time_compiled_encoder(oracle, k, n, stripes):
    """(k, n) without a library-built encoder: compiled by hiprtc from the
    same header text (waited for here), then bit-exact vs the oracle, for all
    pieces and parity only, batched over 3 segments.  RS(37,50) needs two
    input chunks; RS(36,40) is the largest single chunk; RS(3,70) and
    RS(2,98) (96 parity rows, the limit) have more parity rows than 4 compute
    waves hold (the 8 + 4 full encoder).  Before it is ready the same calls run the
    runtime-matrix kernel (test_encode_rebuild_vs_oracle covers that path)."""
    ess = 256
    sch = scheme(k, n, ess)
    # the compiled encoder runs for few parity rows only with the jump-table body selected
    # (otherwise the parity plan's straight-line code does; both checked below)
    assert sch._lib.ec_set_body(sch._ctx, _native.EC_BODY_JUMP_TABLE) == 0
    assert sch._lib.ec_prepare_encoder(sch._ctx, 1) == 1
    assert _kernel_name(sch) == "special-jit"
    rng = np.random.default_rng(k * 7 + n)
    nseg = 3
    seg = rng.integers(0, 256, nseg * stripes * k * ess, dtype=np.uint8)
    f = oracle.FEC(k, n)
    refs = [f.encode_segment(seg[i * stripes * k * ess:(i + 1) * stripes * k * ess], ess, threads=8)
            for i in range(nseg)]
    for body in (_native.EC_BODY_JUMP_TABLE, _native.EC_BODY_STRAIGHT_LINE):
        assert sch._lib.ec_set_body(sch._ctx, body) == 0
        if body == _native.EC_BODY_STRAIGHT_LINE:
            assert _kernel_name(sch) == "straight-line"
        got = gpu_encode(sch, seg, nseg=nseg).cpu().numpy()
        par = gpu_encode(sch, seg, nseg=nseg, parity_only=True).cpu().numpy()
        for i in range(nseg):
            assert np.array_equal(got[i], refs[i]), (body, i)
            assert np.array_equal(par[i], refs[i][k:]), (body, i)


def test_prepare_encoder_reports_limits():
    # n - k > 96 parity rows: outside the compile-time encoder (runtime-matrix kernel)
    sch = scheme(7, 200, 256)
    assert sch._lib.ec_prepare_encoder(sch._ctx, 0) == 0
    assert _kernel_name(sch) == "generic"
    # k > 48: the two-chunk compiled body is no faster than the runtime-matrix kernel there
    s3 = scheme(60, 80, 256)
    assert s3._lib.ec_prepare_encoder(s3._ctx, 0) == 0
    assert _kernel_name(s3) == "straight-line"  # 20 parity rows
    assert s3._lib.ec_set_body(s3._ctx, _native.EC_BODY_JUMP_TABLE) == 0
    assert _kernel_name(s3) == "generic"
    s2 = scheme(29, 80, 256)
    assert s2._lib.ec_prepare_encoder(s2._ctx, 0) == 1


# ---- whole-segment Decode with error detection (ec_decode_segments) -----------

def gpu_decode_segments(sch, d_pieces, nums, stripes):
    k, ess = sch.fc.k, sch.ess
    plen = stripes * ess
    base = d_pieces.data_ptr()
    out = torch.full((stripes * k * ess,), 0xCD, dtype=torch.uint8, device="cuda")
    eestream.SegmentCodec(sch).decode_segments(nums, [base + i * plen for i in nums], stripes, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("k,n,ess,stripes,extras", [
    (29, 80, 256, 9040, (1, 4, 20)),     # the production segment, k+1 .. k+n/4 shares
    (20, 50, 1024, 41, (1, 12)), (30, 60, 256, 130, (2, 15)), (50, 80, 256, 33, (3, 20)), (2, 4, 1024, 7, (1, 2)),
    (4, 10, 256, 1025, (6,)), (3, 5, 100, 4, (2,)),   # ess % 16 != 0: the workspace path
])
def test_decode_segments_clean(oracle, k, n, ess, stripes, extras):
    """Clean pieces, more than k of them in any order: the syndrome check
    finds nothing and the output is the segment (the reference benchmark's
    Decode shape, rs_test.go:616-631, on whole segments)."""
    rng = np.random.default_rng(k * 31 + n + stripes)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    d_pieces = torch.from_numpy(ref).cuda().reshape(1, n, -1)
    for extra in extras:
        nums = [int(x) for x in rng.permutation(n)[:k + extra]]
        assert np.array_equal(gpu_decode_segments(sch, d_pieces, nums, stripes), seg), (k, n, extra)
    assert np.array_equal(d_pieces.cpu().numpy()[0], ref)  # clean pieces are left as they are


@pytest.mark.parametrize("case", ["one bad piece", "scattered", "bad piece + scattered", "too many", "k+1 with error"])
def test_decode_segments_corrects_like_the_oracle(oracle, case):
    """Corrupted pieces through ec_decode_segments: the output and the
    corrected pieces match the oracle's Decode of the same shares (per-stripe
    infectious semantics: Berlekamp-Welch per byte column), and the error
    cases raise what Decode raises."""
    k, n, ess, stripes = 29, 80, 256, 300
    rng = np.random.default_rng(hash(case) % 1000)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    sch = scheme(k, n, ess)
    f = oracle.FEC(k, n)
    ref = f.encode_segment(seg, ess, threads=8)
    extra = 1 if case == "k+1 with error" else 8
    nums = [int(x) for x in rng.permutation(n)[:k + extra]]
    recv = ref.copy()
    plen = stripes * ess
    if case in ("one bad piece", "bad piece + scattered", "too many"):
        recv[nums[3]] ^= rng.integers(1, 256, plen, dtype=np.uint8)
    if case in ("scattered", "bad piece + scattered", "k+1 with error"):
        for t in range(3):
            where = rng.choice(plen, 50, replace=False)
            recv[nums[10 + t]][where] ^= rng.integers(1, 256, 50, dtype=np.uint8)
    if case == "too many":  # 5 > e = 4 bad pieces
        for i in (5, 7, 9, 11):
            recv[nums[i]] ^= rng.integers(1, 256, plen, dtype=np.uint8)
    d_pieces = torch.from_numpy(recv).cuda().reshape(1, n, -1)
    if case in ("too many", "k+1 with error"):
        with pytest.raises(eestream.InfectiousError):
            gpu_decode_segments(sch, d_pieces, nums, stripes)
        with pytest.raises(oracle.OracleError):
            f.decode(sorted(nums), [recv[i].copy() for i in sorted(nums)])
        return
    got = gpu_decode_segments(sch, d_pieces, nums, stripes)
    assert np.array_equal(got, seg)
    fixed = d_pieces.cpu().numpy()[0]
    for i in nums:  # corrected in place
        assert np.array_equal(fixed[i], ref[i]), i
    # the oracle decodes the same received shares to the same bytes: as one long share
    # per piece (columns are independent codewords), its output is the k data pieces
    sn = sorted(nums)
    want = f.decode(sn, [recv[i].copy() for i in sn]).reshape(k, plen)
    assert np.array_equal(want, ref[:k])


def test_decode_segments_batched(oracle):
    """Several segments per call (one check and one rebuild launch): clean
    segments decode; a segment with a bad piece among clean ones is corrected
    on its own, the others untouched."""
    k, n, ess, stripes, nseg = 29, 80, 256, 200, 4
    rng = np.random.default_rng(99)
    sch = scheme(k, n, ess)
    f = oracle.FEC(k, n)
    segs = rng.integers(0, 256, (nseg, stripes * k * ess), dtype=np.uint8)
    refs = np.stack([f.encode_segment(s, ess, threads=8) for s in segs])
    plen = stripes * ess
    nums = [int(x) for x in rng.permutation(n)[:k + 6]]
    for bad_seg in (None, 2):
        recv = refs.copy()
        if bad_seg is not None:
            recv[bad_seg, nums[4]] ^= rng.integers(1, 256, plen, dtype=np.uint8)
        d_pieces = torch.from_numpy(recv).cuda()
        out = torch.zeros((nseg, stripes * k * ess), dtype=torch.uint8, device="cuda")
        base = d_pieces.data_ptr()
        eestream.SegmentCodec(sch).decode_segments(nums, [base + i * plen for i in nums], stripes, out, nseg=nseg,
                                                   piece_seg_stride=n * plen, out_seg_stride=stripes * k * ess)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), segs)
        assert np.array_equal(d_pieces.cpu().numpy(), refs)  # the bad piece corrected in place


def test_auto_body_fresh_share_sets_recycle_plan_memory(oracle):
    """EC_BODY_AUTO with a new share set per call, past the 64 cached plans:
    each set's first launch on the jump table (share-set pass), the next on
    generated code once the background builder has made it; evicted plans
    return their tables to the context's arena, and the recycled memory serves
    the next plans (every result checked)."""
    k, n, ess, stripes = 5, 12, 256, 512
    sch = scheme(k, n, ess)
    rng = np.random.default_rng(92)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    d_pieces = gpu_encode(sch, seg)
    import itertools
    sets = [list(c) for c in itertools.combinations(range(n), k) if any(x >= k for x in c)]
    rng.shuffle(sets)
    for nums in sets[:150]:
        for want in (_native.EC_BODY_JUMP_TABLE, _native.EC_BODY_STRAIGHT_LINE):
            if want == _native.EC_BODY_STRAIGHT_LINE:
                assert prepare_code(sch, nums) == 1
            assert np.array_equal(gpu_rebuild(sch, d_pieces, nums, stripes)[0], seg), nums
            assert sch._lib.ec_last_body(sch._ctx) == want


def test_encode_single_split_batches_keep_each_request_outcome(oracle, monkeypatch):
    """when a coalesced EncodeSingle batch cannot get its
    staging it is split in halves, and every request must come back with the
    outcome of the launch that carried it.  Fault hook (UPLINK_EC_FAULT_SINGLE,
    read at ec_create): batches of more than one request find no staging, and
    neither does a one-request batch for share 5.  So every call for share 5
    fails with EC_ERR_DEVICE and every other call succeeds with the oracle's
    bytes, however the concurrent calls were grouped."""
    k, n, ess = 29, 80, 256
    monkeypatch.setenv("UPLINK_EC_FAULT_SINGLE", "max=1,num=5")
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(k, n, ess, ctypes.byref(ctx)) == 0
    f = oracle.FEC(k, n)
    rng = np.random.default_rng(5)
    stripe = rng.integers(0, 256, k * ess, dtype=np.uint8)
    errors = []

    def work(t):
        out = np.zeros(ess, dtype=np.uint8)
        for rep in range(20):
            num = (t * 7 + rep * 3) % 12  # shares 0..11: data rows, share 5 among them
            out[:] = 0
            rc = L.ec_encode_single(ctx, stripe.ctypes.data, stripe.size, out.ctypes.data, ess, num)
            if num == 5:
                if rc != _native.EC_ERR_DEVICE:
                    errors.append(("share 5 not failed", t, rep, rc))
            elif rc != 0 or not np.array_equal(out, f.encode_single(stripe, num)):
                errors.append(("wrong", t, rep, num, rc))
    try:
        th = [threading.Thread(target=work, args=(t,)) for t in range(24)]
        [t.start() for t in th]
        [t.join() for t in th]
    finally:
        L.ec_destroy(ctx)
    assert not errors, errors[:5]


def test_encoder_queue_reused_across_streams(oracle):
    """The compile-time encoder's work counters are zeroed by each launch's
    last workgroup, not by a memset before the next launch (VERDICT r3 item
    1a).  Launches alternate between three streams and the default stream, many
    more launches than counter slots, some back to back on one stream and some
    handed between streams; every launch's pieces against the oracle."""
    k, n, ess, stripes = 29, 80, 256, 300
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(k, n, ess, ctypes.byref(ctx)) == 0
    f = oracle.FEC(k, n)
    rng = np.random.default_rng(77)
    segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(3)]
    refs = [f.encode_segment(s, ess) for s in segs]
    d_segs = [torch.from_numpy(s).cuda() for s in segs]
    streams = [torch.cuda.Stream() for _ in range(3)] + [torch.cuda.default_stream()]
    try:
        for rnd in range(12):
            outs = []
            for i in range(8):
                st = streams[(rnd + i // 2) % len(streams)]
                d = torch.full((n, stripes * ess), 0xEE, dtype=torch.uint8, device="cuda")
                torch.cuda.current_stream().synchronize()
                assert L.ec_encode_segments(ctx, d_segs[i % 3].data_ptr(), 1, stripes, d.data_ptr(), 0,
                                            st.cuda_stream) == 0
                outs.append((i % 3, d, st))
            for j, d, st in outs:
                st.synchronize()
                assert np.array_equal(d.cpu().numpy(), refs[j]), f"round {rnd}"
    finally:
        torch.cuda.synchronize()
        L.ec_destroy(ctx)


def test_encoder_queue_survives_many_short_lived_streams(oracle):
    """A stream that encodes a few times and goes away (a stream per request)
    does not keep a work-counter slot from the others: 48 streams,
    more than the 32 slots, each encoding twice and then dropped; later
    launches still take a slot (ec_encoder_queue_stats), and every result
    matches the oracle."""
    k, n, ess, stripes = 29, 80, 256, 96
    L = _native.load()
    ctx = ctypes.c_void_p()
    assert L.ec_create(k, n, ess, ctypes.byref(ctx)) == 0
    rng = np.random.default_rng(48)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    ref = oracle.FEC(k, n).encode_segment(seg, ess)
    d_seg = torch.from_numpy(seg).cuda()
    try:
        for i in range(48):
            st = torch.cuda.Stream()
            for _ in range(2):
                d = torch.empty((n, stripes * ess), dtype=torch.uint8, device="cuda")
                assert L.ec_encode_segments(ctx, d_seg.data_ptr(), 1, stripes, d.data_ptr(), 0, st.cuda_stream) == 0
                st.synchronize()
                assert np.array_equal(d.cpu().numpy(), ref), i
            del st
        q, s = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        assert L.ec_encoder_queue_stats(ctx, ctypes.byref(q), ctypes.byref(s)) == 0
        assert q.value + s.value == 96
        assert s.value == 0, (q.value, s.value)  # every launch found a slot
    finally:
        torch.cuda.synchronize()
        L.ec_destroy(ctx)


@pytest.mark.parametrize("body", ["jt", "sl"])
def test_decode_segments_fused_pass_every_shape(oracle, body):
    """The fused Decode launch: rebuilt data rows stored,
    syndrome rows checked for zero, present data shares copied, all in one
    pass over the shares -- under both bodies, for every data share present
    (m = 0: copies and syndromes only), all of them missing (29 rows + the
    syndromes), k+1 and k+n/4 shares, a row count needing several passes of
    the jump-table kernel (29 + 40), and a corrupted piece that the check must
    catch and the per-segment path correct."""
    k, n, ess, stripes = 29, 80, 256, 400
    sch = scheme(k, n, ess)
    want = _native.EC_BODY_JUMP_TABLE if body == "jt" else _native.EC_BODY_STRAIGHT_LINE
    assert sch._lib.ec_set_body(sch._ctx, want) == 0
    rng = np.random.default_rng(4)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    d_pieces = torch.from_numpy(ref).cuda().reshape(1, n, -1)
    sets = [list(range(0, k + 1)), list(range(0, k + 20)), list(range(n - k - 1, n)), list(range(n - k - 20, n)),
            list(range(n - k - 40, n)), [int(x) for x in rng.permutation(n)[:k + 7]]]
    for nums in sets:
        assert np.array_equal(gpu_decode_segments(sch, d_pieces, nums, stripes), seg), nums[:3]
        assert sch._lib.ec_last_body(sch._ctx) == want
    recv = ref.copy()
    nums = list(range(n - k - 8, n))
    recv[nums[2]] ^= rng.integers(1, 256, stripes * ess, dtype=np.uint8)
    d_bad = torch.from_numpy(recv).cuda().reshape(1, n, -1)
    assert np.array_equal(gpu_decode_segments(sch, d_bad, nums, stripes), seg)
    assert np.array_equal(d_bad.cpu().numpy()[0][nums[2]], ref[nums[2]])


def test_decode_segments_wide_code_more_than_128_shares(oracle):
    """Decode of a wide code given more than 128 shares
    checks and corrects every share, as infectious' Correct does
    (private/eestream/rs.go:32-38): RS(100,200) from all 200 shares --
      * clean;
      * one corrupted share past the 128th (outside the one-pass launch's
        inputs: caught by the further syndrome launches, corrected in place);
      * 30 corrupted shares (e = 50 over 200 shares corrects them; over the
        first 128 alone, e = 14 could not);
      * scattered errors in a few columns of many shares;
    every output and every corrected share against the oracle (its Decode and
    its encode), and 51 bad shares: TooManyErrors."""
    k, n, ess, stripes = 100, 200, 256, 8
    sch = scheme(k, n, ess)
    rng = np.random.default_rng(200)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    f = oracle.FEC(k, n)
    ref = f.encode_segment(seg, ess, threads=8)
    nums = [int(x) for x in rng.permutation(n)]
    d_pieces = torch.from_numpy(ref).cuda().reshape(1, n, -1)
    assert np.array_equal(gpu_decode_segments(sch, d_pieces, nums, stripes), seg)
    srt = sorted(nums)

    def corrupt(bad, cols=None):
        recv = ref.copy()
        for i, b in enumerate(bad):
            if cols is None:
                recv[b] ^= rng.integers(1, 256, stripes * ess, dtype=np.uint8)
            else:
                recv[b, cols[i % len(cols)]] ^= 0x3C
        return recv
    for bad, cols in (([srt[150]], None), (sorted(rng.choice(n, 30, replace=False).tolist()), None),
                      (srt[::7], [3, 700, 1500])):
        recv = corrupt(bad, cols)
        # the oracle's Decode of the same shares, stripe by stripe (infectious' Correct + Rebuild)
        want = np.concatenate([f.decode(nums, [recv[x, s * ess:(s + 1) * ess] for x in nums]) for s in range(stripes)])
        assert np.array_equal(want, seg)
        d_bad = torch.from_numpy(recv).cuda().reshape(1, n, -1)
        assert np.array_equal(gpu_decode_segments(sch, d_bad, nums, stripes), want), bad[:4]
        assert np.array_equal(d_bad.cpu().numpy()[0], ref), bad[:4]  # every bad share corrected in place
    recv = corrupt(sorted(rng.choice(n, 51, replace=False).tolist()))
    d_bad = torch.from_numpy(recv).cuda().reshape(1, n, -1)
    with pytest.raises(Exception, match="too many errors"):
        gpu_decode_segments(sch, d_bad, nums, stripes)


def test_decode_host_wide_code_all_shares(oracle):
    """ec_decode (the per-stripe ErasureScheme.Decode) of a wide code: 200
    shares, 40 of them bad, corrected in place against the oracle."""
    k, n, ess = 100, 200, 64
    sch = scheme(k, n, ess)
    rng = np.random.default_rng(201)
    stripe = rng.integers(0, 256, k * ess, dtype=np.uint8)
    f = oracle.FEC(k, n)
    allsh = f.encode(stripe)
    bad = sorted(rng.choice(n, 40, replace=False).tolist())
    shares = [eestream.Share(i, np.array(allsh[i])) for i in range(n)]
    for b in bad:
        shares[b].data[rng.integers(0, ess)] ^= 0x77
    out = sch.decode(None, shares)
    assert np.array_equal(out, stripe)
    for sh in shares:
        assert np.array_equal(sh.data, allsh[sh.number]), sh.number
