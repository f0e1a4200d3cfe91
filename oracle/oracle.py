"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by uplink_amd/).

ctypes binding of oracle/infectious_oracle.c (the CPU restatement of
storj.io/infectious v0.0.2).  Used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, only as the checker or the reported baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libinfectious_oracle.so")

_lib = None

ERRORS = {
    -1: "num must be non-negative",
    -2: "num must be less than {n}",
    -3: "input length must be a multiple of {k}",
    -4: "output length must be {bs}",
    -10: "not enough shares",
    -11: "invalid share id",
    -12: "singular matrix",
    -13: "too many errors to reconstruct",
    -14: "must specify at least one share",
}


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.or_new_fec.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p]
        L.or_lagrange_fec.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.or_encode_single.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, ctypes.c_size_t, u8p,
                                       ctypes.c_size_t, ctypes.c_int]
        L.or_encode.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p, ctypes.c_size_t, u8p]
        L.or_rebuild.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(u8p), ctypes.c_size_t, u8p]
        L.or_decode.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(u8p), ctypes.c_size_t, u8p]
        L.or_decode_fast.argtypes = L.or_decode.argtypes
        L.or_baseline_encode_segment.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, u8p,
                                                 ctypes.c_size_t, u8p, ctypes.c_int]
        L.or_baseline_rebuild_segment.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int,
                                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(u8p),
                                                  ctypes.c_size_t, u8p, ctypes.c_int]
        L.or_fast_encode_segment.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, u8p,
                                             ctypes.c_size_t, u8p, ctypes.c_int]
        L.or_fast_rebuild_segment.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p,
                                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(u8p),
                                              ctypes.c_size_t, u8p, ctypes.c_int]
        L.or_pad.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t]
        L.or_pad.restype = ctypes.c_size_t
        L.or_get_simd.restype = ctypes.c_int
        L.or_set_simd.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class OracleError(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def _err(code: int, **kw) -> OracleError:
    return OracleError(code, ERRORS.get(code, f"error {code}").format(**kw))


def new_fec(k: int, n: int):
    """(enc_matrix n x k, vand_matrix k x n) from the zfec construction."""
    enc = np.zeros(n * k if n * k > 0 else 1, dtype=np.uint8)
    vand = np.zeros(n * k if n * k > 0 else 1, dtype=np.uint8)
    rc = lib().or_new_fec(k, n, _p(enc), _p(vand))
    if rc:
        raise ValueError("requires 1 <= k <= n <= 256")
    return enc[: n * k].reshape(n, k), vand[: n * k].reshape(k, n)


def lagrange_fec(k: int, n: int) -> np.ndarray:
    enc = np.zeros(n * k, dtype=np.uint8)
    if lib().or_lagrange_fec(k, n, _p(enc)):
        raise ValueError("requires 1 <= k <= n <= 256")
    return enc.reshape(n, k)


class FEC:
    """Restatement of infectious.FEC (the *FEC eestream wraps, fec.go:15-17)."""

    def __init__(self, k: int, n: int):
        self.k, self.n = k, n
        self.enc, self.vand = new_fec(k, n)
        self.enc = np.ascontiguousarray(self.enc)

    def encode_single(self, stripe: np.ndarray, num: int) -> np.ndarray:
        stripe = np.ascontiguousarray(stripe, dtype=np.uint8)
        bs = len(stripe) // self.k if self.k else 0
        out = np.zeros(max(bs, 1), dtype=np.uint8)
        rc = lib().or_encode_single(self.k, self.n, _p(self.enc), _p(stripe), len(stripe), _p(out), bs, num)
        if rc:
            raise _err(rc, n=self.n, k=self.k, bs=bs)
        return out[:bs]

    def encode(self, data: np.ndarray) -> np.ndarray:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if len(data) % self.k:
            raise _err(-3, k=self.k)
        bs = len(data) // self.k
        out = np.zeros((self.n, max(bs, 1)), dtype=np.uint8)
        rc = lib().or_encode(self.k, self.n, _p(self.enc), _p(data), len(data), _p(out))
        if rc:
            raise _err(rc, n=self.n, k=self.k, bs=bs)
        return out[:, :bs]

    def _shares_args(self, nums, datas):
        ns = len(nums)
        carr = (ctypes.c_int * max(ns, 1))(*nums)
        keep = [np.ascontiguousarray(d, dtype=np.uint8) for d in datas]
        parr = (ctypes.POINTER(ctypes.c_uint8) * max(ns, 1))(*[_p(d) for d in keep])
        return ns, carr, parr, keep

    def rebuild(self, nums, datas) -> np.ndarray:
        """Returns the k data shares (k, len) in number order."""
        ln = len(datas[0]) if datas else 0
        ns, carr, parr, keep = self._shares_args(nums, datas)
        out = np.zeros((self.k, max(ln, 1)), dtype=np.uint8)
        rc = lib().or_rebuild(self.k, self.n, _p(self.enc), ns, carr, parr, ln, _p(out))
        if rc:
            raise _err(rc)
        return out[:, :ln]

    def decode(self, nums, datas) -> np.ndarray:
        """Correct + Rebuild; returns k*len bytes (unsafe_rs.go:38-46 layout)."""
        if not datas:
            raise _err(-10)
        ln = len(datas[0])
        ns, carr, parr, keep = self._shares_args(nums, [np.array(d, dtype=np.uint8) for d in datas])
        out = np.zeros(self.k * max(ln, 1), dtype=np.uint8)
        rc = lib().or_decode(self.k, self.n, _p(self.enc), ns, carr, parr, ln, _p(out))
        if rc:
            raise _err(rc)
        return out[: self.k * ln]

    def decode_fast(self, nums, datas) -> np.ndarray:
        """Decode as infectious runs it on whole buffers (syndrome rows by addmul,
        Berlekamp-Welch on flagged columns only): the CPU baseline of the
        reference benchmark's Decode; same results as decode()."""
        if not datas:
            raise _err(-10)
        ln = len(datas[0])
        ns, carr, parr, keep = self._shares_args(nums, [np.array(d, dtype=np.uint8) for d in datas])
        out = np.zeros(self.k * max(ln, 1), dtype=np.uint8)
        rc = lib().or_decode_fast(self.k, self.n, _p(self.enc), ns, carr, parr, ln, _p(out))
        if rc:
            raise _err(rc)
        return out[: self.k * ln]

    # segment-level helpers (reference-shaped loops) -----------------------
    def encode_segment(self, seg: np.ndarray, ess: int, threads: int = 1) -> np.ndarray:
        seg = np.ascontiguousarray(seg, dtype=np.uint8)
        stripes = len(seg) // (self.k * ess)
        assert stripes * self.k * ess == len(seg)
        pieces = np.empty((self.n, stripes * ess), dtype=np.uint8)
        lib().or_baseline_encode_segment(self.k, self.n, ess, _p(self.enc), _p(seg), stripes, _p(pieces), threads)
        return pieces

    def rebuild_segment(self, nums, pieces, ess: int, threads: int = 1) -> np.ndarray:
        stripes = len(pieces[0]) // ess
        ns, carr, parr, keep = self._shares_args(list(nums), pieces)
        out = np.empty(stripes * self.k * ess, dtype=np.uint8)
        rc = lib().or_baseline_rebuild_segment(self.k, self.n, ess, _p(self.enc), ns, carr, parr, stripes,
                                               _p(out), threads)
        if rc:
            raise _err(rc)
        return out

    # the optimised CPU variant (all rows per block of stripes; one inversion per share set)
    def fast_encode_segment(self, seg: np.ndarray, ess: int, threads: int = 1) -> np.ndarray:
        seg = np.ascontiguousarray(seg, dtype=np.uint8)
        stripes = len(seg) // (self.k * ess)
        assert stripes * self.k * ess == len(seg)
        pieces = np.empty((self.n, stripes * ess), dtype=np.uint8)
        lib().or_fast_encode_segment(self.k, self.n, ess, _p(self.enc), _p(seg), stripes, _p(pieces), threads)
        return pieces

    def fast_rebuild_segment(self, nums, pieces, ess: int, threads: int = 1) -> np.ndarray:
        """rebuild from exactly k pieces"""
        nums = list(nums)
        assert len(nums) == self.k
        stripes = len(pieces[0]) // ess
        keep = [np.ascontiguousarray(p, dtype=np.uint8) for p in pieces]
        carr = (ctypes.c_int * self.k)(*nums)
        parr = (ctypes.POINTER(ctypes.c_uint8) * self.k)(*[_p(p) for p in keep])
        out = np.empty(stripes * self.k * ess, dtype=np.uint8)
        rc = lib().or_fast_rebuild_segment(self.k, self.n, ess, _p(self.enc), carr, parr, stripes, _p(out), threads)
        if rc:
            raise _err(rc)
        return out


def pad(data: np.ndarray, block: int) -> np.ndarray:
    p = 4 + (block - (len(data) + 4) % block) % block
    buf = np.empty(len(data) + p, dtype=np.uint8)
    buf[: len(data)] = data
    lib().or_pad(_p(buf), len(data), block)
    return buf
