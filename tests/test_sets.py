"""GPU parity of the share-set calls (include/uplink_ec.h
ec_rebuild_segments_sets / ec_decode_segments_sets): many segments in one
pass, each decoded from its own share set, the way concurrent downloads
arrive (private/eestream/stripe.go:314-354 picks whichever k pieces answered
first for every segment; private/ecclient/client.go:273-308; several segments
at once under prefetch, private/storage/streams/store.go:240-253).  Every
output against the segment the oracle encoded; Decode's in-place correction
against the oracle's pieces."""
import ctypes
import os
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from uplink_amd import _native  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


class Ctx:
    def __init__(self, k, n, ess):
        self.L = _native.load()
        self.k, self.n, self.ess = k, n, ess
        self.ctx = ctypes.c_void_p()
        assert self.L.ec_create(k, n, ess, ctypes.byref(self.ctx)) == 0

    def close(self):
        torch.cuda.synchronize()
        self.L.ec_destroy(self.ctx)


def encode_all(oracle, k, n, ess, segs):
    """pieces [nseg, n, plen] on the device, encoded by the oracle"""
    f = oracle.FEC(k, n)
    return torch.from_numpy(np.stack([f.encode_segment(s, ess, threads=8) for s in segs])).cuda()


def call_sets(c, d_pieces, sets, stripes, decode=False, stream=None, outs=None):
    """sets[g] = share numbers of segment g (its pieces: d_pieces[g])"""
    plen = stripes * c.ess
    nseg = len(sets)
    if outs is None:
        outs = torch.full((nseg, stripes * c.k * c.ess), 0xCD, dtype=torch.uint8, device="cuda")
    nsh = (ctypes.c_int * nseg)(*[len(s) for s in sets])
    flat = [x for s in sets for x in s]
    nums = (ctypes.c_int * len(flat))(*flat)
    ptrs = (ctypes.c_void_p * len(flat))(*[d_pieces[g].data_ptr() + x * plen for g, s in enumerate(sets) for x in s])
    optr = (ctypes.c_void_p * nseg)(*[outs[g].data_ptr() for g in range(nseg)])
    st = (stream or torch.cuda.current_stream()).cuda_stream
    fn = c.L.ec_decode_segments_sets if decode else c.L.ec_rebuild_segments_sets
    rc = fn(c.ctx, nseg, nsh, nums, ptrs, stripes, optr, st)
    return rc, outs


def random_sets(rng, k, n, count, extra=0):
    return [[int(x) for x in rng.permutation(n)[:k + extra]] for _ in range(count)]


@pytest.mark.parametrize("k,n,stripes", [(29, 80, 41), (29, 80, 1), (20, 60, 130), (50, 80, 9), (4, 10, 257),
                                          (1, 3, 20), (2, 4, 33)])
def test_rebuild_sets_distinct_set_per_segment(oracle, k, n, stripes):
    """32 segments, 32 different share sets in one call: all parity (the most
    rows), all data present (no rows), seeded random 29-subsets (a mix of
    wave-count classes in one call), sets given in any order and with more
    than k shares; ragged last tile (41 stripes = 5.1 tiles)."""
    ess, nseg = 256, 32
    rng = np.random.default_rng(k * 100 + stripes)
    segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(nseg)]
    d_pieces = encode_all(oracle, k, n, ess, segs)
    sets = [list(range(n - k, n)), list(range(k)), list(range(k))[::-1]]
    sets += random_sets(rng, k, n, nseg - len(sets) - 4)
    sets += random_sets(rng, k, n, 4, extra=min(5, n - k))
    c = Ctx(k, n, ess)
    try:
        rc, outs = call_sets(c, d_pieces, sets, stripes)
        assert rc == 0, _native.strerror(rc)
        torch.cuda.synchronize()
        got = outs.cpu().numpy()
        for g in range(nseg):
            assert np.array_equal(got[g], segs[g]), (g, sets[g][:6])
        assert c.L.ec_last_body(c.ctx) == _native.EC_BODY_JUMP_TABLE
    finally:
        c.close()


def test_rebuild_sets_full_size_and_limits(oracle):
    """A production RS(29,80) 64 MiB segment (9040 stripes) with a fresh set
    next to a small one in the same call; and RS(128,256), the engine's limit:
    128 inputs, up to 128 rows in 4 passes of 32."""
    k, n, ess = 29, 80, 256
    rng = np.random.default_rng(9040)
    raw = rng.integers(0, 256, 64 * 2**20, dtype=np.uint8)
    seg = oracle.pad(raw, k * ess)
    stripes = seg.size // (k * ess)
    d_pieces = encode_all(oracle, k, n, ess, [seg, seg])
    c = Ctx(k, n, ess)
    try:
        sets = [sorted(rng.choice(n, k, replace=False).tolist()), list(range(n - k, n))]
        rc, outs = call_sets(c, d_pieces, sets, stripes)
        assert rc == 0
        torch.cuda.synchronize()
        assert np.array_equal(outs[0].cpu().numpy(), seg) and np.array_equal(outs[1].cpu().numpy(), seg)
    finally:
        c.close()
    k, n, stripes = 128, 256, 3
    segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(3)]
    d_pieces = encode_all(oracle, k, n, ess, segs)
    c = Ctx(k, n, ess)
    try:
        sets = [list(range(128, 256)), sorted(rng.choice(n, k, replace=False).tolist()),
                list(range(28)) + list(range(156, 256))]
        rc, outs = call_sets(c, d_pieces, sets, stripes)
        assert rc == 0
        torch.cuda.synchronize()
        for g in range(3):
            assert np.array_equal(outs[g].cpu().numpy(), segs[g]), g
    finally:
        c.close()


@pytest.mark.parametrize("one", [1, 0])
def test_rebuild_sets_one_segment(oracle, one):
    """One segment per call (configs[2] as a single download runs it): one
    launch with the rows solved on the host (rs_sets_one), or --
    UPLINK_EC_SETS_ONE=0 -- the prep launch and the pass.  Full-size
    RS(29,80) from all parity and from a random set; RS(128,256) (4 passes of
    32 rows on 4 waves, past the one-launch limits: the two launches);
    RS(40,100) (40 rows: 2 passes in one launch); RS(1,3);
    all data present (no rows); a ragged last tile; one-segment calls
    alternating on one context with many-segment calls (the slot's completion
    counter each leaves at zero)."""
    os.environ["UPLINK_EC_SETS_ONE"] = str(one)
    try:
        rng = np.random.default_rng(2 + one)
        k, n, ess = 29, 80, 256
        seg = oracle.pad(rng.integers(0, 256, 64 * 2**20, dtype=np.uint8), k * ess)
        stripes = seg.size // (k * ess)
        d_pieces = encode_all(oracle, k, n, ess, [seg])
        c = Ctx(k, n, ess)
        try:
            for s in (list(range(n - k, n)), sorted(rng.choice(n, k, replace=False).tolist()), list(range(k))):
                rc, outs = call_sets(c, d_pieces, [s], stripes)
                assert rc == 0, _native.strerror(rc)
                torch.cuda.synchronize()
                assert np.array_equal(outs[0].cpu().numpy(), seg), s[:4]
        finally:
            c.close()
        for k, n, stripes in ((128, 256, 3), (40, 100, 7), (1, 3, 20), (29, 80, 41), (20, 60, 130)):
            segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(3)]
            d_pieces = encode_all(oracle, k, n, ess, segs)
            c = Ctx(k, n, ess)
            try:
                for it in range(6):
                    sets = random_sets(rng, k, n, 3, extra=it % 2)
                    if it % 3 == 2:
                        sets[0] = list(range(n - k, n))
                    pick = [it % 3] if it % 2 == 0 else [0, 1, 2]
                    rc, outs = call_sets(c, d_pieces[pick[0]:pick[-1] + 1], [sets[g] for g in pick], stripes)
                    assert rc == 0, _native.strerror(rc)
                    torch.cuda.synchronize()
                    got = outs.cpu().numpy()
                    for i, g in enumerate(pick):
                        assert np.array_equal(got[i], segs[g]), (k, n, it, g)
            finally:
                c.close()
    finally:
        os.environ.pop("UPLINK_EC_SETS_ONE", None)


def test_rebuild_sets_errors():
    """Errors as Rebuild reports them, before anything is launched: a segment
    with fewer than k shares, a share number out of range, a share given twice
    among the k chosen."""
    k, n, ess, stripes = 4, 10, 256, 3
    c = Ctx(k, n, ess)
    try:
        d_pieces = torch.zeros((2, n, stripes * ess), dtype=torch.uint8, device="cuda")
        rc, _ = call_sets(c, d_pieces, [[0, 1, 2, 3], [5, 6, 7]], stripes)
        assert rc == _native.EC_ERR_NOT_ENOUGH_SHARES
        rc, _ = call_sets(c, d_pieces, [[0, 1, 2, 3], [5, 6, 7, 10]], stripes)
        assert rc == _native.EC_ERR_INVALID_SHARE
        rc, _ = call_sets(c, d_pieces, [[0, 1, 2, 3], [5, 6, 7, 7]], stripes)
        assert rc == _native.EC_ERR_SINGULAR
        rc, _ = call_sets(c, d_pieces, [], stripes)
        assert rc == 0
    finally:
        c.close()


@pytest.mark.parametrize("nseg", [6, 1])
def test_rebuild_sets_many_calls_streams_and_threads(oracle, nseg):
    """More calls in flight than the context's 16 slots, from 4 threads on 4
    streams: a slot is reused only once the GPU has finished the call that
    used it (its last workgroup's completion word), so every segment of every
    call is rebuilt from its own set.  nseg = 1: every call the one-launch
    pass, whose leaf table lives in the slot too."""
    k, n, ess, stripes = 29, 80, 256, 64
    rng = np.random.default_rng(16 + nseg)
    segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(nseg)]
    d_pieces = encode_all(oracle, k, n, ess, segs)
    c = Ctx(k, n, ess)
    errors = []
    try:
        def work(t):
            st = torch.cuda.Stream()
            r = np.random.default_rng(t)
            pending = []
            for call in range(24):
                sets = random_sets(r, k, n, nseg)
                with torch.cuda.stream(st):
                    rc, outs = call_sets(c, d_pieces, sets, stripes, stream=st)
                if rc:
                    errors.append((t, call, rc))
                pending.append(outs)
            st.synchronize()
            for outs in pending:
                got = outs.cpu().numpy()
                for g in range(nseg):
                    if not np.array_equal(got[g], segs[g]):
                        errors.append((t, g))
        th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
        [x.start() for x in th]
        [x.join() for x in th]
    finally:
        c.close()
    assert not errors, errors[:5]


def test_decode_sets_clean_and_corrupted(oracle):
    """Decode with error detection over per-segment sets: clean segments from
    k .. k+20 shares decode in the one pass; a segment with a corrupted piece
    is caught by its syndromes, its piece corrected in place (as infectious
    corrects share.Data) and the segment rebuilt; the others untouched."""
    k, n, ess, stripes, nseg = 29, 80, 256, 40, 8
    rng = np.random.default_rng(407)
    segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(nseg)]
    f = oracle.FEC(k, n)
    refs = np.stack([f.encode_segment(s, ess, threads=8) for s in segs])
    recv = refs.copy()
    sets = [[int(x) for x in rng.permutation(n)[:k + e]] for e in (0, 1, 4, 20, 10, 10, 3, 7)]
    bad_seg, bad_share = 4, sets[4][6]
    recv[bad_seg][bad_share] ^= rng.integers(1, 256, stripes * ess, dtype=np.uint8)
    d_pieces = torch.from_numpy(recv).cuda()
    c = Ctx(k, n, ess)
    try:
        rc, outs = call_sets(c, d_pieces, sets, stripes, decode=True)
        assert rc == 0, _native.strerror(rc)
        got = outs.cpu().numpy()
        for g in range(nseg):
            assert np.array_equal(got[g], segs[g]), g
        assert np.array_equal(d_pieces.cpu().numpy(), refs)  # the bad piece corrected in place
        # more errors than k+20 shares correct (e = 10) in one segment: TooManyErrors
        recv2 = refs.copy()
        for x in sets[3][:15]:
            recv2[3][x] ^= 0x5A
        d2 = torch.from_numpy(recv2).cuda()
        rc, _ = call_sets(c, d2, sets, stripes, decode=True)
        assert rc == _native.EC_ERR_TOO_MANY_ERRORS
    finally:
        c.close()


def test_batched_rebuild_fresh_sets_no_host_wait(oracle):
    """ec_rebuild_segments_batched with share sets the context has never seen
    runs the share-set pass (the jump-table body); the set's straight-line code
    is made in the background and taken by a later launch.  Results bit-exact
    either way."""
    k, n, ess, stripes = 29, 80, 256, 600
    rng = np.random.default_rng(600)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    d_pieces = encode_all(oracle, k, n, ess, [seg])
    c = Ctx(k, n, ess)
    plen = stripes * ess
    try:
        for _ in range(6):
            nums = sorted(rng.choice(n, k, replace=False).tolist())
            out = torch.empty(stripes * k * ess, dtype=torch.uint8, device="cuda")
            cn = (ctypes.c_int * k)(*nums)
            cp = (ctypes.c_void_p * k)(*[d_pieces[0].data_ptr() + i * plen for i in nums])
            st = torch.cuda.current_stream().cuda_stream
            assert c.L.ec_rebuild_segments_batched(c.ctx, k, cn, cp, stripes, 1, 0, 0, out.data_ptr(), st) == 0
            assert c.L.ec_last_body(c.ctx) == _native.EC_BODY_JUMP_TABLE
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), seg)
            assert c.L.ec_prepare_rebuild(c.ctx, k, cn, 1) == 1
            assert c.L.ec_rebuild_segments_batched(c.ctx, k, cn, cp, stripes, 1, 0, 0, out.data_ptr(), st) == 0
            assert c.L.ec_last_body(c.ctx) == _native.EC_BODY_STRAIGHT_LINE
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), seg)
    finally:
        c.close()


def test_segment_codec_sets_host_mirror(oracle):
    """The host mirror's SegmentCodec.rebuild_segments_sets /
    decode_segments_sets (eestream.py) over the same exports: segments from
    share sets of their own, one of them with a corrupted piece for Decode,
    the errors Rebuild reports raised as the mirror's exceptions."""
    from uplink_amd import eestream as E

    k, n, ess, stripes, nseg = 20, 60, 256, 33, 6
    rng = np.random.default_rng(2060)
    segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(nseg)]
    f = oracle.FEC(k, n)
    refs = np.stack([f.encode_segment(s, ess, threads=8) for s in segs])
    scheme = E.new_rs_scheme(E.new_fec(k, n), ess)
    codec = E.SegmentCodec(scheme)
    try:
        d_pieces = torch.from_numpy(refs.copy()).cuda()
        plen = stripes * ess
        sets = random_sets(rng, k, n, nseg, extra=3)
        args = [(st, [d_pieces[g].data_ptr() + x * plen for x in st]) for g, st in enumerate(sets)]
        outs = torch.zeros((nseg, stripes * k * ess), dtype=torch.uint8, device="cuda")
        codec.rebuild_segments_sets(args, stripes, [outs[g] for g in range(nseg)])
        torch.cuda.synchronize()
        got = outs.cpu().numpy()
        assert all(np.array_equal(got[g], segs[g]) for g in range(nseg))
        bad = sets[2][1]
        recv = refs.copy()
        recv[2][bad] ^= 0x77
        d2 = torch.from_numpy(recv).cuda()
        args2 = [(st, [d2[g].data_ptr() + x * plen for x in st]) for g, st in enumerate(sets)]
        outs.zero_()
        codec.decode_segments_sets(args2, stripes, [outs[g] for g in range(nseg)])
        got = outs.cpu().numpy()
        assert all(np.array_equal(got[g], segs[g]) for g in range(nseg))
        assert np.array_equal(d2.cpu().numpy(), refs)
        with pytest.raises(E.NotEnoughShares):
            codec.rebuild_segments_sets([(sets[0][:k - 1], args[0][1][:k - 1])], stripes, [outs[0]])
        with pytest.raises(ValueError):
            codec.rebuild_segments_sets(args, stripes, [outs[0]])
    finally:
        torch.cuda.synchronize()
        scheme.close()


@pytest.mark.parametrize("decode", [False, True])
def test_sets_segments_off_the_bit_sliced_path(oracle, decode):
    """Segments the share-set pass cannot take go through the single-set paths
    inside the same call, with the same results: a share size that is not a
    multiple of 16 (the byte kernel), and, at ess 256, one segment whose
    output and one whose piece is not 16-byte aligned, beside aligned ones."""
    rng = np.random.default_rng(100 + decode)
    for k, n, ess, stripes in [(4, 10, 100, 37), (29, 80, 256, 9)]:
        nseg = 4
        segs = [rng.integers(0, 256, stripes * k * ess, dtype=np.uint8) for _ in range(nseg)]
        plen = stripes * ess
        f = oracle.FEC(k, n)
        refs = np.stack([f.encode_segment(s, ess, threads=8) for s in segs])
        # pieces and outputs in buffers 16 bytes longer, so a segment can sit 8 bytes in
        d_pieces = torch.zeros((nseg, n * plen + 16), dtype=torch.uint8, device="cuda")
        outs = torch.zeros((nseg, stripes * k * ess + 16), dtype=torch.uint8, device="cuda")
        pshift = [0, 8, 0, 0] if ess % 16 == 0 else [0] * nseg
        oshift = [0, 0, 8, 0] if ess % 16 == 0 else [0] * nseg
        for g in range(nseg):
            d_pieces[g, pshift[g]:pshift[g] + n * plen] = torch.from_numpy(refs[g].reshape(-1)).cuda()
        sets = random_sets(rng, k, n, nseg, extra=2 if decode else 0)
        c = Ctx(k, n, ess)
        try:
            nsh = (ctypes.c_int * nseg)(*[len(s) for s in sets])
            flat = [x for s in sets for x in s]
            nums = (ctypes.c_int * len(flat))(*flat)
            ptrs = (ctypes.c_void_p * len(flat))(
                *[d_pieces[g].data_ptr() + pshift[g] + x * plen for g, s in enumerate(sets) for x in s])
            optr = (ctypes.c_void_p * nseg)(*[outs[g].data_ptr() + oshift[g] for g in range(nseg)])
            fn = c.L.ec_decode_segments_sets if decode else c.L.ec_rebuild_segments_sets
            rc = fn(c.ctx, nseg, nsh, nums, ptrs, stripes, optr, torch.cuda.current_stream().cuda_stream)
            assert rc == 0, _native.strerror(rc)
            torch.cuda.synchronize()
            got = outs.cpu().numpy()
            for g in range(nseg):
                assert np.array_equal(got[g, oshift[g]:oshift[g] + stripes * k * ess], segs[g]), (k, ess, g)
        finally:
            c.close()


def test_decode_sets_one_segment(oracle):
    """One segment (its record passed in the prep launch's arguments) through
    Decode: clean from k+3 shares, then with a corrupted piece, corrected in
    place as infectious corrects share.Data."""
    k, n, ess, stripes = 29, 80, 256, 50
    rng = np.random.default_rng(1)
    seg = rng.integers(0, 256, stripes * k * ess, dtype=np.uint8)
    ref = oracle.FEC(k, n).encode_segment(seg, ess, threads=8)
    st = [int(x) for x in rng.permutation(n)[:k + 3]]
    c = Ctx(k, n, ess)
    try:
        d = torch.from_numpy(ref[None].copy()).cuda()
        rc, outs = call_sets(c, d, [st], stripes, decode=True)
        assert rc == 0, _native.strerror(rc)
        assert np.array_equal(outs[0].cpu().numpy(), seg)
        bad = ref[None].copy()
        bad[0][st[2]] ^= 0x3C
        d2 = torch.from_numpy(bad).cuda()
        rc, outs = call_sets(c, d2, [st], stripes, decode=True)
        assert rc == 0, _native.strerror(rc)
        assert np.array_equal(outs[0].cpu().numpy(), seg)
        assert np.array_equal(d2.cpu().numpy()[0], ref)
    finally:
        c.close()
