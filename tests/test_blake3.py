"""BLAKE3 piece hashing: the CPU oracle against the
official test vectors, and (gpu) the engine's kernel against the oracle.

Reference path: private/piecestore/hash.go:20-26 (BLAKE3 is the default
PieceHashAlgorithm), upload.go:133 (NewHashFromAlgorithm), :155 (TeeReader
over the piece bytes), :270 (Hash: Sum(nil)).
"""
import json
import os

import numpy as np
import pytest

from oracle import blake3 as ob

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "blake3_vectors.json")


def _pattern(n):
    return (np.arange(n) % 251).astype(np.uint8)


def _vectors():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("n,want", _vectors()["vectors"])
def test_oracle_official_vectors(n, want):
    assert ob.blake3(_pattern(n)).hex() == want


def test_oracle_strings():
    for s, want in _vectors()["strings"]:
        assert ob.blake3(s.encode()).hex() == want


def test_oracle_many_matches_single():
    rng = np.random.default_rng(3)
    pieces = rng.integers(0, 256, (7, 5000), dtype=np.uint8)
    many = ob.blake3_many(pieces, threads=3)
    for i in range(7):
        assert many[i].tobytes() == ob.blake3(pieces[i])


# ---------------------------------------------------------------- GPU ----

def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
def test_gpu_official_vectors():
    """The kernel itself against the published vectors (one launch, every length)."""
    _gpu()
    from uplink_amd import piecehash
    for n, want in _vectors()["vectors"]:
        assert piecehash.blake3_host(_pattern(n))[0].tobytes().hex() == want, n


# lengths around every boundary: block (64), chunk (1024), workgroup group
# (256 chunks), one parents level (65536 chunks) and the BASELINE piece
LENGTHS = [0, 1, 63, 64, 65, 1000, 1023, 1024, 1025, 2047, 2048, 2049, 3 * 1024 + 7, 255 * 1024, 256 * 1024 - 1,
           256 * 1024, 256 * 1024 + 1, 257 * 1024, 511 * 1024 + 64, 512 * 1024 + 1024, 1 << 20, 2314240, 2319360]


@pytest.mark.gpu
@pytest.mark.parametrize("ln", LENGTHS)
def test_gpu_matches_oracle(ln):
    _gpu()
    from uplink_amd import piecehash
    rng = np.random.default_rng(ln)
    pieces = rng.integers(0, 256, (3, ln), dtype=np.uint8)
    assert np.array_equal(piecehash.blake3_host(pieces), ob.blake3_many(pieces, threads=3))


@pytest.mark.gpu
def test_gpu_two_parent_levels():
    """> 65536 chunks: the parents kernel runs twice (257 groups -> 2 -> root)."""
    _gpu()
    from uplink_amd import piecehash
    rng = np.random.default_rng(9)
    for ln in (64 * 1024 * 1024 + 1025, 64 * 1024 * 1024):
        a = rng.integers(0, 256, ln, dtype=np.uint8)
        assert piecehash.blake3_host(a)[0].tobytes() == ob.blake3(a), ln


@pytest.mark.gpu
@pytest.mark.parametrize("run,gap,offset", [(256, 7424 - 256, 0), (1024, 4096, 16), (100, 60, 0), (256, 256, 1),
                                            (64, 0, 0)])
def test_gpu_strided_views(run, gap, offset):
    """Pieces made of runs (the data pieces inside a stripe-major segment),
    unaligned bases and non power-of-two runs (byte path)."""
    torch = _gpu()
    from uplink_amd import piecehash
    rng = np.random.default_rng(run + gap + offset)
    npieces, nruns = 5, 37
    run_stride = run + gap
    piece_len = nruns * run - 13  # ragged last run
    piece_stride = nruns * run_stride + 32
    buf = rng.integers(0, 256, offset + npieces * piece_stride + run_stride, dtype=np.uint8)
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(npieces * 32, dtype=torch.uint8, device="cuda")
    piecehash.blake3_device(d.data_ptr() + offset, npieces, piece_len, piece_stride, out, run=run,
                            run_stride=run_stride)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(npieces, 32)
    for j in range(npieces):
        p0 = offset + j * piece_stride
        ref = np.concatenate([buf[p0 + r * run_stride:p0 + r * run_stride + run] for r in range(nruns)])[:piece_len]
        assert got[j].tobytes() == ob.blake3(ref), j


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,ess,stripes", [(29, 80, 256, 9040), (4, 10, 256, 300), (2, 4, 1024, 1), (3, 7, 100, 50),
                                             (1, 1, 256, 9), (20, 60, 4096, 40)])
def test_gpu_segment_hashes(k, n, ess, stripes):
    """ec_hash_segments / ec_encode_segments_host_hashed: the hash of every
    piece (data pieces read in place from the segment) against the oracle's
    hash of the oracle's pieces."""
    torch = _gpu()
    from oracle import oracle as O
    from uplink_amd import eestream, piecehash
    sch = eestream.RSScheme(eestream.new_fec(k, n), ess)
    rng = np.random.default_rng(k * n + stripes)
    nseg = 2
    segs = rng.integers(0, 256, nseg * stripes * k * ess, dtype=np.uint8)
    fec = O.FEC(k, n)
    want = np.stack([ob.blake3_many(fec.encode_segment(segs.reshape(nseg, -1)[s], ess, threads=8), threads=8)
                     for s in range(nseg)])
    # device form
    d_segs = torch.from_numpy(segs).cuda()
    d_par = torch.empty((nseg, n - k, stripes * ess), dtype=torch.uint8, device="cuda")
    if n > k:
        eestream.SegmentCodec(sch).encode_segments(d_segs, nseg, stripes, d_par, parity_only=True)
    d_h = torch.zeros((nseg, n, 32), dtype=torch.uint8, device="cuda")
    piecehash.hash_segments(sch, d_segs, d_par if n > k else None, nseg, stripes, d_h)
    torch.cuda.synchronize()
    assert np.array_equal(d_h.cpu().numpy(), want)
    # host pipeline form, both output layouts
    from uplink_amd import _native as N
    for flags, rows in ((0, n), (N.EC_FLAG_PARITY_ONLY, n - k)):
        pieces = np.zeros((nseg, rows, stripes * ess), dtype=np.uint8)
        hashes = np.zeros((nseg, n, 32), dtype=np.uint8)
        rc = N.load().ec_encode_segments_host_hashed(sch.ctx, segs.ctypes.data, nseg, stripes, pieces.ctypes.data,
                                                     hashes.ctypes.data, flags)
        assert rc == 0
        assert np.array_equal(hashes, want)
        ref = np.stack([fec.encode_segment(segs.reshape(nseg, -1)[s], ess, threads=8) for s in range(nseg)])
        assert np.array_equal(pieces, ref[:, n - rows:])


@pytest.mark.gpu
def test_segment_piece_reader_hashes():
    """SegmentPieceReader(hash_pieces=True).piece_hash(num) == BLAKE3 of the
    bytes piece_reader(num) streams (what upload.go:155,270 would hash)."""
    _gpu()
    from uplink_amd import eestream, segment
    rs = eestream.new_redundancy_strategy(eestream.RSScheme(eestream.new_fec(29, 80), 256), 0, 0)
    data = np.random.default_rng(5).integers(0, 256, 3 * 1024 * 1024 + 77, dtype=np.uint8).tobytes()
    r = segment.SegmentPieceReader(data, rs, hash_pieces=True)
    try:
        for num in (0, 5, 28, 29, 50, 79):
            assert r.piece_hash(num) == ob.blake3(r.piece_reader(num).read()), num
    finally:
        r.close()
