"""Host logic of the eestream mirror and the C-ABI surface (no GPU needed)."""
import ctypes
import os
import re

import pytest

from uplink_amd import _native, eestream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Scheme:
    """Duck-typed ErasureScheme (sizes only) for host-logic tests."""

    def __init__(self, k, n, ess):
        self.k, self.n, self.ess = k, n, ess

    def total_count(self):
        return self.n

    def required_count(self):
        return self.k

    def stripe_size(self):
        return self.k * self.ess

    def erasure_share_size(self):
        return self.ess


@pytest.mark.parametrize("rep,opt,exp_rep,exp_opt,err", [
    # rs_test.go:155-190 (TestNewRedundancyStrategy), RS(2,4)
    (0, 0, 4, 4, ""),
    (-1, 0, 0, 0, "eestream: negative repair threshold"),
    (1, 0, 0, 0, "eestream: repair threshold less than required count"),
    (5, 0, 0, 0, "eestream: repair threshold greater than total count"),
    (0, -1, 0, 0, "eestream: negative optimal threshold"),
    (0, 1, 0, 0, "eestream: optimal threshold less than required count"),
    (0, 5, 0, 0, "eestream: optimal threshold greater than total count"),
    (3, 4, 3, 4, ""),
    (0, 3, 0, 0, "eestream: repair threshold greater than optimal threshold"),
    (4, 3, 0, 0, "eestream: repair threshold greater than optimal threshold"),
    (4, 4, 4, 4, ""),
])
def test_new_redundancy_strategy(rep, opt, exp_rep, exp_opt, err):
    es = _Scheme(2, 4, 8 * 1024)
    if err:
        with pytest.raises(eestream.EEStreamError) as ei:
            eestream.RedundancyStrategy(es, rep, opt)
        assert str(ei.value) == err
    else:
        rs = eestream.RedundancyStrategy(es, rep, opt)
        assert (rs.repair_threshold(), rs.optimal_threshold()) == (exp_rep, exp_opt)


@pytest.mark.parametrize("size,expected", [(0, 1024), (1, 1024), (1020, 1024), (1024, 1024), (32764, 16384),
                                           (32768, 17408), (32868, 17408)])
def test_calc_piece_size(size, expected):
    assert eestream.calc_piece_size(size, _Scheme(2, 4, 1024)) == expected


def test_pad_unpad_roundtrip():
    for n in (0, 1, 7423, 7424, 7425, 100000):
        data = os.urandom(n)
        p = eestream.pad(data, 7424)
        assert len(p) % 7424 == 0 and len(p) - n >= 4
        assert eestream.unpad(p) == data
    # the synthetic 64 MiB segment pads to 9040 stripes
    assert (64 * 2**20 + 4 + 7423) // 7424 == 9040


def _header_functions():
    with open(os.path.join(ROOT, "include", "uplink_ec.h")) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ec_[a-z_]+)\s*\(", text)))


def test_library_exports_every_header_symbol(native):
    names = _header_functions()
    assert len(names) >= 18
    for name in names:
        assert hasattr(native, name), name
        assert name in _native.SIGNATURES, name


def test_error_strings_match_reference(native):
    assert native.ec_strerror(_native.EC_ERR_NUM_NEGATIVE).decode() == "num must be non-negative"
    buf = ctypes.create_string_buffer(64)
    native.ec_format_error(None, _native.EC_ERR_NUM_RANGE, 4, buf, 64)
    assert buf.value.decode() == "num must be less than 4"
    assert native.ec_strerror(_native.EC_ERR_PARAMS).decode() == "requires 1 <= k <= n <= 256"


def test_create_rejects_bad_params(native):
    h = ctypes.c_void_p()
    for k, n in [(0, 4), (5, 4), (1, 257)]:
        assert native.ec_create(k, n, 256, ctypes.byref(h)) == _native.EC_ERR_PARAMS


def test_no_cpu_fallback_without_gpu(native):
    """Without a HIP device the product refuses to run (no silent CPU path)."""
    if native.ec_device_count() > 0:
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    assert native.ec_create(29, 80, 256, ctypes.byref(h)) == _native.EC_ERR_DEVICE
    with pytest.raises(eestream.DeviceError):
        eestream.RSScheme(eestream.new_fec(29, 80), 256)


def test_adjacent_stage_entry_points_validate_before_the_device(native):
    """The BLAKE3 / AES-GCM / padding exports reject bad arguments (and accept
    empty work) without touching a device, like the RS exports."""
    assert native.ec_gcm_key_bytes() >= 60 * 4 + 64 * 16 * 16
    assert native.ec_blake3_pieces(None, 0, 0, 0, 0, 0, None, None) == _native.EC_ERR_INVALID_ARG  # no output
    out = ctypes.create_string_buffer(32)
    assert native.ec_blake3_pieces(None, 0, 0, 0, 0, 0, out, None) == _native.EC_OK  # nothing to hash
    assert native.ec_blake3_pieces(None, 1, 0, 10, 0, 0, out, None) == _native.EC_ERR_INVALID_ARG
    assert native.ec_gcm_prepare_keys(None, 0, None, None) == _native.EC_OK
    assert native.ec_gcm_prepare_keys(None, 1, None, None) == _native.EC_ERR_INVALID_ARG
    assert native.ec_gcm_seal_segments(None, 1, 1, 7408, None, None, None, None) == _native.EC_ERR_INVALID_ARG
    assert native.ec_gcm_seal_segments(None, 0, 1, 7408, None, None, None, None) == _native.EC_OK
    assert native.ec_gcm_open_segments(None, 1, 1, 7408, None, None, None, None, None) == _native.EC_ERR_INVALID_ARG
    assert native.ec_gcm_seal_host(None, None, None, 0, 7408, None) == _native.EC_ERR_INVALID_ARG
    assert native.ec_pad_segments(None, 1, 0, 10, 16, None) == _native.EC_ERR_INVALID_ARG
    assert native.ec_pad_segments(None, 0, 0, 10, 16, None) == _native.EC_OK
    assert native.ec_strerror(_native.EC_ERR_AUTH).decode() == "cipher: message authentication failed"
