"""The measurement exports and the share-set calls' guard rails on the GPU:
ec_encode_shape_probe (the RS(29,80) encoder's schedule without its
arithmetic, bench.py's on-box ceiling: the data pieces copied through for
real, every parity row a copy of the tile's last input share), and a
share-set call on a capturing stream refused before anything is staged
(its completion words need the launches to run)."""
import ctypes

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


def _ctx(L, k, n, ess=256):
    c = ctypes.c_void_p()
    assert L.ec_create(k, n, ess, ctypes.byref(c)) == 0
    return c


@pytest.mark.parametrize("nseg,stripes", [(1, 9040), (3, 257), (2, 1)])
def test_encode_shape_probe_moves_the_encoders_bytes(nseg, stripes):
    L = _native.load()
    k, n, ess = 29, 80, 256
    ctx = _ctx(L, k, n, ess)
    try:
        plen = stripes * ess
        g = torch.Generator(device="cuda")
        g.manual_seed(nseg * 1000 + stripes)
        segs = torch.randint(0, 256, (nseg, stripes * k * ess), dtype=torch.uint8, device="cuda", generator=g)
        sp = torch.cuda.current_stream().cuda_stream
        full = torch.zeros((nseg, n, plen), dtype=torch.uint8, device="cuda")
        assert L.ec_encode_shape_probe(ctx, segs.data_ptr(), nseg, stripes, full.data_ptr(), 0, sp) == 0
        par = torch.zeros((nseg, n - k, plen), dtype=torch.uint8, device="cuda")
        assert L.ec_encode_shape_probe(ctx, segs.data_ptr(), nseg, stripes, par.data_ptr(),
                                       _native.EC_FLAG_PARITY_ONLY, sp) == 0
        torch.cuda.synchronize()
        shares = segs.view(nseg, stripes, k, ess).permute(0, 2, 1, 3).reshape(nseg, k, plen)
        assert torch.equal(full[:, :k], shares)  # the copy-through is the encoder's own
        last = shares[:, k - 1:k].expand(nseg, n - k, plen)
        assert torch.equal(full[:, k:], last)  # each parity row: the tile's last input
        assert torch.equal(par, last)
    finally:
        L.ec_destroy(ctx)


def test_encode_shape_probe_other_codes_unsupported():
    L = _native.load()
    ctx = _ctx(L, 20, 60)
    try:
        buf = torch.zeros(60 * 256 * 4, dtype=torch.uint8, device="cuda")
        assert L.ec_encode_shape_probe(ctx, buf.data_ptr(), 1, 2, buf.data_ptr(), 0, None) == \
            _native.EC_ERR_UNSUPPORTED
    finally:
        L.ec_destroy(ctx)


def test_sets_call_refused_under_stream_capture():
    L = _native.load()
    k, n, ess, stripes = 4, 10, 256, 16
    ctx = _ctx(L, k, n, ess)
    try:
        pieces = torch.zeros((n, stripes * ess), dtype=torch.uint8, device="cuda")
        out = torch.zeros(stripes * k * ess, dtype=torch.uint8, device="cuda")
        nums = list(range(n - k, n))
        s = torch.cuda.Stream()
        graph = torch.cuda.CUDAGraph()
        rc = None
        with torch.cuda.graph(graph, stream=s, capture_error_mode="relaxed"):
            torch.zeros(1, device="cuda")  # (something for the graph to hold)
            rc = L.ec_rebuild_segments_sets(ctx, 1, (ctypes.c_int * 1)(k), (ctypes.c_int * k)(*nums),
                                            (ctypes.c_void_p * k)(*[pieces[j].data_ptr() for j in nums]), stripes,
                                            (ctypes.c_void_p * 1)(out.data_ptr()), ctypes.c_void_p(s.cuda_stream))
        assert rc == _native.EC_ERR_UNSUPPORTED
        # the context still works afterwards, on a plain stream
        rc = L.ec_rebuild_segments_sets(ctx, 1, (ctypes.c_int * 1)(k), (ctypes.c_int * k)(*nums),
                                        (ctypes.c_void_p * k)(*[pieces[j].data_ptr() for j in nums]), stripes,
                                        (ctypes.c_void_p * 1)(out.data_ptr()), None)
        assert rc == 0
        torch.cuda.synchronize()
    finally:
        L.ec_destroy(ctx)
