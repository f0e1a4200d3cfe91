"""AES-256-GCM segment encryption: the CPU oracle
against the GCM specification's test cases and storj's framing rules, and
(gpu) the engine's kernels against the oracle.

Reference path: splitter/splitter.go:156 NewEncrypter(EncAESGCM, key, nonce,
BlockSize = 29*256 (project.go:84)), :170 TransformWriterPadded;
streams/store.go:347-382 decryptRanger (NewDecrypter, Transform, Unpad);
nonces splitter/common.go:27-32, store.go:264-270.
"""
import json
import os

import numpy as np
import pytest

from oracle import aesgcm as oa
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "aesgcm_vectors.json")


def _cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("c", _cases(), ids=lambda c: c["name"])
def test_oracle_gcm_spec_vectors(c):
    k, iv, aad, pt = (bytes.fromhex(c[x]) for x in ("key", "iv", "aad", "pt"))
    sealed = oa.seal(k, iv, pt, aad)
    assert sealed.hex() == c["ct"] + c["tag"]
    if not aad:
        assert oa.open_(k, iv, sealed) == pt


def test_nonce_increment_little_endian():
    assert oa.increment(bytes(12), 1) == b"\x01" + bytes(11)
    assert oa.increment(b"\xff" + bytes(11), 1) == b"\x00\x01" + bytes(10)
    assert oa.increment(bytes(12), 0x0102030405) == bytes([5, 4, 3, 2, 1]) + bytes(7)
    # nonceForPosition: PartNumber<<32 | Index+1 (splitter/common.go:29)
    assert oa.nonce_for_position(0, 0) == b"\x01" + bytes(23)
    assert oa.nonce_for_position(2, 7) == bytes([8, 0, 0, 0, 2]) + bytes(19)


def test_segment_sizes_match_reference():
    """64 MiB plaintext -> 9059 blocks of 7424 = standardMaxEncryptedSegmentSize
    (buffer/backend.go:20)."""
    in_block = 29 * 256 - 16
    p = 4 + (in_block - (64 * 2**20 + 4) % in_block) % in_block
    assert (64 * 2**20 + p) // in_block == 9059
    assert 9059 * 29 * 256 == 67254016


def test_oracle_segment_round_trip_and_tamper():
    rng = np.random.default_rng(1)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonce = oa.nonce_for_position(0, 3)
    plain = rng.integers(0, 256, 50000, dtype=np.uint8).tobytes()
    enc = oa.encrypt_segment(plain, key, nonce, threads=3)
    assert len(enc) % (29 * 256) == 0
    assert oa.decrypt_segment(enc, key, nonce, len(plain), threads=2) == plain
    bad = bytearray(enc)
    bad[29 * 256 + 5] ^= 1  # second block
    assert oa.decrypt_segment(bytes(bad), key, nonce, len(plain)) is None
    # block b is sealed under nonce + b
    blk = 29 * 256 - 16
    padded = O.pad(np.frombuffer(plain, dtype=np.uint8), blk)
    b = 4
    assert enc[b * 7424:(b + 1) * 7424].tobytes() == oa.seal(key, oa.increment(nonce[:12], b),
                                                            padded[b * blk:(b + 1) * blk].tobytes())


def test_host_mirror_nonce_matches_oracle():
    from uplink_amd import encryption as E
    for part, idx in ((0, 0), (1, 2), (7, 1 << 20), (0xFFFF, 0xFFFFFFFE)):
        assert E.nonce_for_position(part, idx) == oa.nonce_for_position(part, idx)
    assert E.increment(b"\xff" * 12, 1) == bytes(12)


# ---------------------------------------------------------------- GPU ----

def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("c", [c for c in _cases() if not c["aad"] and c["pt"] and len(c["pt"]) % 32 == 0],
                         ids=lambda c: c["name"])
def test_gpu_gcm_spec_vectors(c):
    """GCM test cases 14 and 15 (16-byte-multiple plaintext, no AAD) as one
    block each, straight through the kernel."""
    _gpu()
    from uplink_amd import _native as N
    k, iv, pt = (bytes.fromhex(c[x]) for x in ("key", "iv", "pt"))
    out = np.zeros(len(pt) + 16, dtype=np.uint8)
    p = np.frombuffer(pt, dtype=np.uint8).copy()
    assert N.load().ec_gcm_seal_host(k, iv, p.ctypes.data, 1, len(pt), out.ctypes.data) == 0
    assert out.tobytes().hex() == c["ct"] + c["tag"]


@pytest.mark.gpu
@pytest.mark.parametrize("in_block", [16, 48, 992, 1008, 1024, 1040, 2032, 4080, 7408])
def test_gpu_blocks_match_oracle(in_block):
    """Block sizes around the 64-lane slot padding (63, 64, 65 sub-blocks +
    the length block), storj's 7408, and small ones."""
    _gpu()
    from uplink_amd import encryption as E
    rng = np.random.default_rng(in_block)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonce = rng.integers(0, 256, 24, dtype=np.uint8).tobytes()
    nb = 37
    padded = rng.integers(0, 256, nb * in_block, dtype=np.uint8)
    got = E.AESGCMEncrypter(key, nonce, in_block + 16).transform(padded)
    want = oa.encrypt_blocks(key, nonce, padded, in_block, threads=4).reshape(-1)
    assert got == want.tobytes()
    back = E.AESGCMDecrypter(key, nonce, in_block + 16).transform(got)
    assert back == padded.tobytes()


@pytest.mark.gpu
def test_gpu_nonce_carry():
    """Starting nonces whose low bytes overflow within the segment: the
    little-endian increment must carry (calcGCMNonce)."""
    _gpu()
    from uplink_amd import encryption as E
    rng = np.random.default_rng(2)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    for nonce in (b"\xf0" + b"\xff" * 7 + bytes(4), b"\xff" * 12, bytes(11) + b"\x80"):
        padded = rng.integers(0, 256, 300 * 7408, dtype=np.uint8)
        got = E.AESGCMEncrypter(key, nonce, 7424).transform(padded)
        assert got == oa.encrypt_blocks(key, nonce, padded, 7408, threads=8).reshape(-1).tobytes()


@pytest.mark.gpu
def test_gpu_segment_round_trip_and_tamper():
    """A full 64 MiB plaintext segment: TransformWriterPadded equivalent is
    bit-exact with the oracle (9059 blocks = standardMaxEncryptedSegmentSize);
    decryption restores it; a flipped ciphertext or tag bit fails
    authentication on that block."""
    _gpu()
    from uplink_amd import encryption as E
    rng = np.random.default_rng(7)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    nonce = E.nonce_for_position(0, 5)
    plain = rng.integers(0, 256, 64 * 2**20, dtype=np.uint8).tobytes()
    enc = E.encrypt_segment(plain, key, nonce)
    assert len(enc) == 67254016
    assert enc == oa.encrypt_segment(plain, key, nonce, threads=16).tobytes()
    assert E.decrypt_segment(enc, key, nonce, len(plain)) == plain
    assert E.decrypt_segment(enc, key, nonce) == plain  # Unpad from the trailer
    for pos, blk in ((7424 * 1000 + 17, 1000), (7424 * 9059 - 1, 9058), (7424 * 5 + 7408, 5)):
        bad = bytearray(enc)
        bad[pos] ^= 0x10
        with pytest.raises(E.DecryptionFailed) as ei:
            E.decrypt_segment(bytes(bad), key, nonce, len(plain))
        assert ei.value.block == blk
    with pytest.raises(E.DecryptionFailed):  # wrong key
        E.decrypt_segment(enc, bytes(32), nonce, len(plain))


@pytest.mark.gpu
def test_gpu_batched_segments_device():
    """ec_gcm_seal_segments / ec_gcm_open_segments over a batch of segments
    with their own keys and nonces, device-resident; per-segment status."""
    torch = _gpu()
    from uplink_amd import encryption as E
    rng = np.random.default_rng(11)
    nseg, nb, ib = 5, 123, 7408
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(nseg)]
    nonces = [E.nonce_for_position(1, i) for i in range(nseg)]
    plain = rng.integers(0, 256, (nseg, nb * ib), dtype=np.uint8)
    d_plain = torch.from_numpy(plain).cuda()
    d_keys = E.prepare_keys(keys)
    d_nonces = torch.from_numpy(np.frombuffer(b"".join(n[:12] for n in nonces), dtype=np.uint8).copy()).cuda()
    d_ct = torch.empty((nseg, nb * (ib + 16)), dtype=torch.uint8, device="cuda")
    E.seal_segments(d_plain, nseg, nb, ib, d_keys, d_nonces, d_ct)
    torch.cuda.synchronize()
    ct = d_ct.cpu().numpy()
    for g in range(nseg):
        assert np.array_equal(ct[g], oa.encrypt_blocks(keys[g], nonces[g], plain[g], ib, threads=8).reshape(-1))
    d_ct[2, 77 * (ib + 16) + 3] ^= 1
    d_pt = torch.empty_like(d_plain)
    d_status = torch.zeros(nseg, dtype=torch.int32, device="cuda")
    E.open_segments(d_ct, nseg, nb, ib, d_keys, d_nonces, d_pt, d_status)
    torch.cuda.synchronize()
    assert d_status.cpu().tolist() == [-1, -1, 77, -1, -1]
    pt = d_pt.cpu().numpy()
    for g in (0, 1, 3, 4):
        assert np.array_equal(pt[g], plain[g])
