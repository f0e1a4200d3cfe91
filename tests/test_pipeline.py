"""The device-resident upload/download chain (uplink_amd/pipeline.py):
encrypt -> PadReader -> RS encode -> BLAKE3, and rebuild -> decrypt, against
the same chain of oracles (storj's AES-GCM framing, infectious, BLAKE3).
Reference: splitter/splitter.go:156,170; segmentupload/single.go:236;
segmentupload/encode.go:39-75; piecestore/upload.go:155,270;
eestream/stripe.go:382-428; streams/store.go:347-382."""
import numpy as np
import pytest

from oracle import aesgcm as oa
from oracle import blake3 as ob
from oracle import oracle as O



def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_geometry_matches_reference_sizes():
    """64 MiB plaintext: 9059 GCM blocks = 67,254,016 B = 9059 stripes, padded
    to 9060 stripes (2,319,360-byte pieces), SURVEY Appendix B."""
    from uplink_amd import pipeline

    class Sizes:  # the two sizes SegmentGeometry reads from an RSScheme (no device needed)
        def stripe_size(self):
            return 29 * 256

        def erasure_share_size(self):
            return 256

    g = pipeline.SegmentGeometry(64 * 2**20, Sizes())
    assert (g.nblocks, g.enc_len, g.nstripes, g.piece_len) == (9059, 67254016, 9060, 2319360)


@pytest.mark.gpu
@pytest.mark.parametrize("k,n,plain_len,nseg", [(29, 80, 64 * 2**20, 2), (29, 80, 100_000, 3), (4, 10, 7407, 2),
                                                (29, 80, 1, 1)])
def test_upload_download_chain(k, n, plain_len, nseg):
    torch = _torch()
    from uplink_amd import eestream, encryption as E, pipeline
    sch = eestream.RSScheme(eestream.new_fec(k, n), 256)
    p = pipeline.DevicePipeline(sch, plain_len)
    g = p.g
    rng = np.random.default_rng(plain_len + k)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(nseg)]
    nonces = [E.nonce_for_position(0, i) for i in range(nseg)]
    plains = [rng.integers(0, 256, plain_len, dtype=np.uint8) for _ in range(nseg)]
    d_plain, d_enc, d_pieces, d_hashes = p.buffers(nseg)
    for i in range(nseg):
        d_plain[i, :plain_len] = torch.from_numpy(plains[i])
    d_keys, d_nonces = p.prepare_keys(keys), p.nonces_tensor(nonces)
    p.upload(d_plain, nseg, d_keys, d_nonces, d_enc, d_pieces, d_hashes)
    torch.cuda.synchronize()
    fec = O.FEC(k, n)
    pieces, hashes = d_pieces.cpu().numpy(), d_hashes.cpu().numpy()
    for i in range(nseg):
        enc = oa.encrypt_segment(plains[i].tobytes(), keys[i], nonces[i], threads=8)
        padded = O.pad(np.frombuffer(enc.tobytes(), dtype=np.uint8), k * 256)
        ref = fec.encode_segment(padded, 256, threads=8)
        assert np.array_equal(pieces[i], ref), i
        assert np.array_equal(hashes[i], ob.blake3_many(ref, threads=8)), i
    # download from the last k pieces (all parity when n >= 2k)
    nums = list(range(n - k, n))
    d_out = torch.zeros((nseg, g.plain_cap), dtype=torch.uint8, device="cuda")
    d_status = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    p.download(nums, d_pieces, nseg, d_keys, d_nonces, d_enc, d_out, d_status)
    torch.cuda.synchronize()
    assert d_status.cpu().tolist() == [-1] * nseg
    out = d_out.cpu().numpy()
    for i in range(nseg):
        assert np.array_equal(out[i, :plain_len], plains[i]), i
    # a corrupted piece byte rebuilds into a corrupted ciphertext block: authentication fails there
    stripe_of_byte = 5 % g.nstripes
    d_pieces[nseg - 1, nums[0], stripe_of_byte * 256 + 3] ^= 0x40
    p.download(nums, d_pieces, nseg, d_keys, d_nonces, d_enc, d_out, d_status)
    torch.cuda.synchronize()
    st = d_status.cpu().tolist()
    assert st[:-1] == [-1] * (nseg - 1)
    # stripe s of the encrypted segment is GCM block s * stripe / 7424 (equal sizes when k = 29)
    assert st[-1] == (stripe_of_byte * k * 256) // 7424 or (stripe_of_byte >= g.nblocks and st[-1] == -1)
