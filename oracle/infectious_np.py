"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by uplink_amd/).

numpy restatement of storj.io/infectious v0.0.2, the GF(2^8) Reed-Solomon
module private/eestream delegates to (go.mod:17; absent from this container).
It is an independent second restatement next to infectious_oracle.c: the C
file follows the zfec inverted-Vandermonde construction, this file builds the
generator from the closed-form Lagrange basis,
and tests/test_oracle.py requires the two to agree byte for byte.

Call sites served (reference file:line):
  new_fec        eestream.NewFEC                private/eestream/fec.go:15-17
  encode_single  rsScheme.EncodeSingle          private/eestream/rs.go:21-23
  encode         rsScheme.Encode                private/eestream/rs.go:25-30
  rebuild        rsScheme.Rebuild               private/eestream/rs.go:40-45
  pad            encryption.PadReader           segmentupload/single.go:236 (storj.io/common)
  calc_piece_size eestream.CalcPieceSize        private/eestream/encode.go:272-281
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D

EXP = np.zeros(510, dtype=np.uint8)
LOG = np.zeros(256, dtype=np.int64)
_x = 1
for _i in range(255):
    EXP[_i] = _x
    EXP[_i + 255] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= POLY
LOG[0] = 255

MUL = np.zeros((256, 256), dtype=np.uint8)
_a = np.arange(1, 256)
MUL[1:, 1:] = EXP[(LOG[_a][:, None] + LOG[_a][None, :])]
INV = np.zeros(256, dtype=np.uint8)
INV[1:] = EXP[255 - LOG[_a]]


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def points(n: int) -> list[int]:
    """Evaluation points x_0 = 0, x_r = a^(r-1) (zfec indexing)."""
    return [0] + [int(EXP[(r - 1) % 255]) for r in range(1, n)]


def new_fec(k: int, n: int) -> np.ndarray:
    """n x k systematic generator G[i][j] = L_j(x_i) (Lagrange basis)."""
    if not (1 <= k <= n <= 256):
        raise ValueError("requires 1 <= k <= n <= 256")
    xs = points(n)
    G = np.zeros((n, k), dtype=np.uint8)
    for i in range(n):
        for j in range(k):
            num, den = 1, 1
            for m in range(k):
                if m == j:
                    continue
                num = gf_mul(num, xs[i] ^ xs[m])
                den = gf_mul(den, xs[j] ^ xs[m])
            G[i, j] = gf_mul(num, int(INV[den]))
    return G


def invert(m: np.ndarray) -> np.ndarray:
    k = m.shape[0]
    a = np.concatenate([m.astype(np.uint8), np.eye(k, dtype=np.uint8)], axis=1)
    for c in range(k):
        nz = np.nonzero(a[c:, c])[0]
        if len(nz) == 0:
            raise ValueError("singular matrix")
        p = c + int(nz[0])
        if p != c:
            a[[c, p]] = a[[p, c]]
        a[c] = MUL[int(INV[a[c, c]])][a[c]]
        for r in range(k):
            if r != c and a[r, c]:
                a[r] ^= MUL[int(a[r, c])][a[c]]
    return a[:, k:].copy()


def matvec_blocks(M: np.ndarray, blocks: np.ndarray) -> np.ndarray:
    """out[i] = XOR_j M[i,j] * blocks[j]  (blocks: (k, L) uint8)."""
    out = np.zeros((M.shape[0], blocks.shape[1]), dtype=np.uint8)
    for i in range(M.shape[0]):
        for j in range(M.shape[1]):
            c = int(M[i, j])
            if c:
                out[i] ^= MUL[c][blocks[j]]
    return out


def encode_single(G: np.ndarray, stripe: bytes | np.ndarray, num: int) -> np.ndarray:
    n, k = G.shape
    if num < 0:
        raise ValueError("num must be non-negative")
    if num >= n:
        raise ValueError(f"num must be less than {n}")
    a = np.frombuffer(bytes(stripe), dtype=np.uint8) if not isinstance(stripe, np.ndarray) else stripe
    if len(a) % k:
        raise ValueError(f"input length must be a multiple of {k}")
    blocks = a.reshape(k, -1)
    if num < k:
        return blocks[num].copy()
    return matvec_blocks(G[num:num + 1], blocks)[0]


def encode_segment(G: np.ndarray, seg: np.ndarray, ess: int) -> np.ndarray:
    """Segment [stripe][k][ess] -> pieces [n][stripes*ess] (every stripe's
    share i appended to piece i, segmentupload/encode.go:39-75)."""
    n, k = G.shape
    stripes = len(seg) // (k * ess)
    cols = seg.reshape(stripes, k, ess).transpose(1, 0, 2).reshape(k, stripes * ess)
    pieces = np.empty((n, stripes * ess), dtype=np.uint8)
    pieces[:k] = cols
    if n > k:
        pieces[k:] = matvec_blocks(G[k:], cols)
    return pieces


def rebuild_segment(G: np.ndarray, nums: list[int], pieces: list[np.ndarray], ess: int) -> np.ndarray:
    """Rebuild from exactly the given shares (front/back selection of
    infectious Rebuild), returning the stripe-major segment."""
    n, k = G.shape
    if len(nums) < k:
        raise ValueError("not enough shares")
    order = sorted(range(len(nums)), key=lambda i: nums[i])
    nums = [nums[i] for i in order]
    pieces = [pieces[i] for i in order]
    b, e = 0, len(nums) - 1
    chosen = []
    for i in range(k):
        if nums[b] == i:
            chosen.append(b)
            b += 1
        else:
            chosen.append(e)
            e -= 1
    ids = [nums[c] for c in chosen]
    D = invert(G[ids])
    data = matvec_blocks(D, np.stack([pieces[c] for c in chosen]))
    stripes = data.shape[1] // ess
    return data.reshape(k, stripes, ess).transpose(1, 0, 2).reshape(-1)


def pad(data: bytes, block: int) -> bytes:
    p = 4 + (block - (len(data) + 4) % block) % block
    tail = bytearray([p & 0xFF] * p)
    tail[-4:] = p.to_bytes(4, "big")
    return bytes(data) + bytes(tail)


def calc_piece_size(data_size: int, k: int, ess: int) -> int:
    stripe = k * ess
    stripes = (data_size + 4 + stripe - 1) // stripe
    return stripes * stripe // k
