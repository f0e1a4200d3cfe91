"""Straight-line rebuild bodies (uplink_amd/csrc/rs_sl_codegen.cpp, DESIGN.md
§4): the code the library generates per decode plan, checked on the CPU
before any of it runs on a GPU.

tests/c/build/sl_dump runs the library's generator on a matrix; the code
words are disassembled by the LLVM disassembler of the ROCm image (an
encoder independent of the library's), and the disassembly is executed by a
small emulator of the five instruction forms against GF(2^8) arithmetic from
the oracle (oracle/infectious_np.py).  Every segment must:
  * use only ds_read_b128 (from v126), s_waitcnt lgkmcnt, v_xor_b32,
    v_bitop3_b32 (0x96), and end in s_setpc_b64 s[48:49];
  * write only its rows' accumulators v[32 + 8o .. 39 + 8o] and the scratch
    v[96:125];
  * wait for every LDS read before its destination is used;
  * leave acc[o] ^= sum_j M[rbase + o][j] * x_j for the chunk's inputs.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import infectious_np as inp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "tests", "c", "build", "sl_dump")
LLVM_MC = "/opt/rocm/lib/llvm/bin/llvm-mc"

pytestmark = pytest.mark.skipif(not (os.path.exists(DUMP) and os.path.exists(LLVM_MC)),
                                reason="sl_dump (tests/c) or llvm-mc missing")

GF_MUL = None


def gf_mul_table():
    global GF_MUL
    if GF_MUL is None:
        t = np.zeros((256, 256), dtype=np.uint8)
        for a in range(256):
            for b in range(256):
                t[a, b] = inp.gf_mul(a, b)
        GF_MUL = t
    return GF_MUL


def generate(M, cap=None):
    rows, nin = M.shape
    text = f"{rows} {nin}\n" + " ".join(str(int(x)) for x in M.reshape(-1)) + "\n"
    cmd = [DUMP] + ([str(cap)] if cap else [])
    out = subprocess.run(cmd, input=text, capture_output=True, text=True, check=True).stdout.splitlines()
    nw, npass, nchunks = map(int, out[0].split()[1:])
    offs = [int(x) for x in out[1].split()[1:]]
    n = int(out[2].split()[1])
    words = [int(x, 16) for x in out[3:3 + n]]
    return nw, npass, nchunks, offs, words


def disassemble(words):
    """LLVM's disassembly of the words, one (mnemonic, operands) per instruction."""
    data = " ".join(f"0x{b:02x}" for w in words for b in w.to_bytes(4, "little"))
    r = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "--disassemble"], input=data, capture_output=True,
                       text=True, check=True)
    assert "invalid" not in r.stderr.lower(), r.stderr
    ins = []
    for line in r.stdout.splitlines():
        line = line.split(";")[0].strip()
        if not line or line.startswith("."):
            continue
        mn, _, ops = line.partition(" ")
        ins.append((mn, ops.strip()))
    return ins


def segment_words(words, off):
    """The words of the segment at byte offset `off`, up to its s_setpc_b64."""
    i = off // 4
    out = []
    while True:
        w = words[i]
        out.append(w)
        if w == 0xBE801D30:  # s_setpc_b64 s[48:49]
            return out
        i += 1


def vreg(s):
    m = re.fullmatch(r"v(\d+)", s.strip())
    assert m, s
    return int(m.group(1))


def busy(pending):
    return {r for t in pending for r in t}


def emulate(ins, lds, acc_rows):
    """Run one segment on one lane: `lds` maps byte offset -> 32-bit plane word,
    v[32 + 8o + p] start at 0.  Returns the accumulators and the registers
    written."""
    v = {}
    for o in range(acc_rows):
        for p in range(8):
            v[32 + 8 * o + p] = 0
    pending = []  # destinations of LDS reads not yet waited for, in issue order
    written = set()
    ended = False
    for mn, ops in ins:
        assert not ended, "instruction after s_setpc_b64"
        if mn == "ds_read_b128":
            m = re.fullmatch(r"v\[(\d+):(\d+)\], v126(?: offset:(\d+))?", ops)
            assert m, ops
            d0, d1, off = int(m.group(1)), int(m.group(2)), int(m.group(3) or 0)
            assert d1 == d0 + 3
            for i in range(4):
                v[d0 + i] = lds[off + 4 * i]
                written.add(d0 + i)
            pending.append(tuple(range(d0, d0 + 4)))
        elif mn == "s_waitcnt":
            m = re.fullmatch(r"lgkmcnt\((\d+)\)", ops)
            assert m, ops
            keep = int(m.group(1))
            pending = pending[len(pending) - keep:] if keep else []
        elif mn in ("v_xor_b32_e32", "v_xor_b32"):
            d, a, b = (vreg(x) for x in ops.split(","))
            assert not {a, b} & busy(pending), "operand used before its LDS read landed"
            v[d] = v[a] ^ v[b]
            written.add(d)
        elif mn == "v_bitop3_b32":
            m = re.fullmatch(r"(v\d+), (v\d+), (v\d+), (v\d+) bitop3:0x96", ops)
            assert m, ops
            d, a, b, c = (vreg(m.group(i)) for i in range(1, 5))
            assert not {a, b, c} & busy(pending)
            v[d] = v[a] ^ v[b] ^ v[c]
            written.add(d)
        elif mn == "s_setpc_b64":
            assert ops == "s[48:49]", ops
            ended = True
        else:
            raise AssertionError(f"unexpected instruction {mn} {ops}")
    assert ended, "segment does not return"
    assert not pending, "LDS read still pending at return"
    return v, written


def planes_of(x):
    """bytes x[32] (one lane's 32 columns) -> 8 planes: plane p bit b = bit p of byte b"""
    return [sum(((int(x[b]) >> p) & 1) << b for b in range(32)) for p in range(8)]


def bytes_of(planes):
    return np.array([sum(((planes[p] >> b) & 1) << p for p in range(8)) for b in range(32)], dtype=np.uint8)


def check_matrix(M, seed):
    rng = np.random.default_rng(seed)
    mul = gf_mul_table()
    rows, nin = M.shape
    nw, npass, nchunks, offs, words = generate(M)
    assert len(offs) == npass * nchunks * nw
    assert 0 < len(words) <= 524288  # the large region
    chs = -(-nin // nchunks)  # chunks dealt evenly (rs_kernels.hip)
    for pass_ in range(npass):
        p0 = pass_ * rows // npass
        prow = (pass_ + 1) * rows // npass - p0
        for ch in range(nchunks):
            j0, jn = ch * chs, min(chs, nin - ch * chs)
            x = rng.integers(0, 256, (jn, 32), dtype=np.uint8)
            lds = {}
            for jj in range(jn):  # the straight-line layout (rs_device.hpp slice_inputs WIDE), lane 0
                for p, w in enumerate(planes_of(x[jj])):
                    lds[jj * 2048 + 1024 * (p // 4) + 4 * (p % 4)] = w
            for g in range(nw):
                rbase = p0 + g * prow // nw
                cnt = p0 + (g + 1) * prow // nw - rbase
                off = offs[(pass_ * nchunks + ch) * nw + g]
                if cnt <= 0:
                    assert off == -1
                    continue
                assert off > 0 and off % 64 == 0
                ins = disassemble(segment_words(words, off))
                v, written = emulate(ins, lds, cnt)
                allowed = set(range(96, 126)) | {32 + 8 * o + p for o in range(cnt) for p in range(8)}
                assert written <= allowed, sorted(written - allowed)
                for o in range(cnt):
                    want = np.zeros(32, dtype=np.uint8)
                    for jj in range(jn):
                        want ^= mul[M[rbase + o, j0 + jj], x[jj]]
                    got = bytes_of([v[32 + 8 * o + p] for p in range(8)])
                    assert np.array_equal(got, want), (pass_, ch, g, o)


def test_rebuild_matrix_all_parity_29_80():
    """The bench's worst case: RS(29,80) from pieces 51..79, 29 rows x 29 inputs."""
    ids = list(range(51, 80))
    G = inp.new_fec(29, 80)
    D = inp.invert(G[ids])
    check_matrix(D, 1)


@pytest.mark.parametrize("rows,nin,zero_frac", [(1, 1, 0.0), (3, 5, 0.3), (16, 29, 0.0), (17, 20, 0.5),
                                                (24, 29, 0.1), (29, 29, 0.9), (33, 7, 0.0), (64, 40, 0.2),
                                                (128, 12, 0.0)])
def test_random_matrices(rows, nin, zero_frac):
    """Every wave count (2, 3, 4), multi-pass row splits, ragged chunks, zero
    and unit coefficients."""
    rng = np.random.default_rng(rows * 1000 + nin)
    M = rng.integers(0, 256, (rows, nin), dtype=np.uint8)
    M[rng.random((rows, nin)) < zero_frac] = 0
    M[rng.random((rows, nin)) < 0.05] = 1
    check_matrix(M, rows + nin)


def test_rows_without_terms():
    """Rows with no nonzero coefficient, or whose first term comes in a later
    chunk, or with a single term."""
    rng = np.random.default_rng(3)
    M = rng.integers(1, 256, (20, 29), dtype=np.uint8)
    M[3] = 0
    M[7, :16] = 0
    M[12, 1:] = 0
    check_matrix(M, 9)


def test_region_sizes():
    """A plan that does not fit the 256-KiB region is refused there
    (generate() returns 0 words) and takes the 2-MiB one: the largest plan,
    128 rows x 128 inputs of nonzero coefficients (two passes of eight
    waves), fits it and computes the right products."""
    rng = np.random.default_rng(5)
    M = rng.integers(1, 256, (128, 128), dtype=np.uint8)
    assert generate(M, cap=65536)[4] == []
    words = generate(M)[4]
    assert 65536 < len(words) <= 524288
    check_matrix(M, 11)


def test_wave_split_by_row_count():
    """The row split the kernel launch and the code generator share (split_for,
    rs_sl_codegen.cpp): 2 waves up to 14 rows, 3 up to 24 (RS(29,80) m = 16
    on 3, DESIGN.md §4 "Rebuild, round 4"), 4 up to 32, 8 past that (one pass
    up to 64 rows, several beyond); chunks of 2 inputs per wave."""
    want = {1: (2, 1), 14: (2, 1), 15: (3, 1), 16: (3, 1), 24: (3, 1), 25: (4, 1), 29: (4, 1), 32: (4, 1),
            33: (8, 1), 40: (8, 1), 64: (8, 1), 65: (8, 2), 128: (8, 2)}
    for rows, (nw, npass) in want.items():
        got = generate(np.ones((rows, 29), dtype=np.uint8))
        assert got[:2] == (nw, npass), rows
        assert got[2] == -(-29 // (2 * nw)), rows  # chunks of at most 2 nw inputs
