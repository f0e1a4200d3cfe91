"""ctypes binding of libuplink_ec.so (include/uplink_ec.h).

The product path: every call below runs on the GPU.  If the shared library is
missing or no GPU is usable the calls raise — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libuplink_ec.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "uplink_ec.h")

EC_OK = 0
EC_ERR_PARAMS = -1
EC_ERR_NUM_NEGATIVE = -2
EC_ERR_NUM_RANGE = -3
EC_ERR_INPUT_LENGTH = -4
EC_ERR_OUTPUT_LENGTH = -5
EC_ERR_NOT_ENOUGH_SHARES = -6
EC_ERR_TOO_MANY_ERRORS = -7
EC_ERR_INVALID_SHARE = -8
EC_ERR_SINGULAR = -9
EC_ERR_INVALID_ARG = -10
EC_ERR_DEVICE = -11
EC_ERR_UNSUPPORTED = -12
EC_ERR_SHARE_SIZE = -13
EC_ERR_AUTH = -14

EC_FLAG_PARITY_ONLY = 0x1
EC_FLAG_HASH_PIECES = 0x2
# ec_set_body: body of the runtime-matrix kernel (include/uplink_ec.h)
EC_BODY_AUTO, EC_BODY_JUMP_TABLE, EC_BODY_STRAIGHT_LINE = 0, 1, 2
# ec_bw_probe shapes
EC_PROBE_COPY, EC_PROBE_ENCODE_MIX, EC_PROBE_PARITY_MIX = 0, 1, 2

u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p

# name -> (restype, argtypes); must list every symbol include/uplink_ec.h declares
SIGNATURES = {
    "ec_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
    "ec_destroy": (None, [vp]),
    "ec_required": (ctypes.c_int, [vp]),
    "ec_total": (ctypes.c_int, [vp]),
    "ec_share_size": (ctypes.c_int, [vp]),
    "ec_stripe_size": (ctypes.c_int, [vp]),
    "ec_generator": (ctypes.c_int, [vp, vp]),
    "ec_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "ec_format_error": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_longlong, ctypes.c_char_p, ctypes.c_size_t]),
    "ec_encode_single": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.c_int]),
    "ec_encode": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp]),
    "ec_rebuild": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                  ctypes.c_size_t, vp]),
    "ec_decode": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                 ctypes.c_size_t, vp]),
    "ec_encode_segments": (ctypes.c_int, [vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, ctypes.c_int, vp]),
    "ec_rebuild_segments": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                           ctypes.c_size_t, vp, vp]),
    "ec_decode_segments": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                          ctypes.c_size_t, vp, vp]),
    "ec_decode_segments_batched": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                                  ctypes.c_size_t, ctypes.c_size_t, ctypes.c_longlong,
                                                  ctypes.c_longlong, vp, vp]),
    "ec_rebuild_segments_batched": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_size_t,
                                                   ctypes.c_longlong, ctypes.c_longlong, vp, vp]),
    "ec_rebuild_segments_sets": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp), ctypes.c_size_t,
                                                ctypes.POINTER(vp), vp]),
    "ec_decode_segments_sets": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp), ctypes.c_size_t,
                                               ctypes.POINTER(vp), vp]),
    "ec_prepare_rebuild": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "ec_encode_segments_host": (ctypes.c_int, [vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, ctypes.c_int]),
    "ec_rebuild_segments_host": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp),
                                                ctypes.c_size_t, ctypes.c_size_t, ctypes.c_longlong, vp]),
    "ec_encode_segments_host_hashed": (ctypes.c_int, [vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, vp,
                                                      ctypes.c_int]),
    "ec_blake3_pieces": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_size_t,
                                        ctypes.c_longlong, vp, vp]),
    "ec_hash_segments": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, vp]),
    "ec_blake3_host": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, ctypes.c_size_t, vp]),
    "ec_gcm_key_bytes": (ctypes.c_size_t, []),
    "ec_gcm_prepare_keys": (ctypes.c_int, [vp, ctypes.c_size_t, vp, vp]),
    "ec_gcm_seal_segments": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, vp, vp, vp, vp]),
    "ec_gcm_open_segments": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, vp, vp, vp, vp,
                                            vp]),
    "ec_gcm_seal_segments_strided": (ctypes.c_int, [vp, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_size_t,
                                                    ctypes.c_size_t, vp, vp, vp, ctypes.c_longlong, vp]),
    "ec_gcm_open_segments_strided": (ctypes.c_int, [vp, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_size_t,
                                                    ctypes.c_size_t, vp, vp, vp, ctypes.c_longlong, vp, vp]),
    "ec_pad_segments": (ctypes.c_int, [vp, ctypes.c_size_t, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_size_t, vp]),
    "ec_gcm_seal_host": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp]),
    "ec_gcm_open_host": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp,
                                        ctypes.POINTER(ctypes.c_longlong)]),
    "ec_upload_begin": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp, ctypes.c_int, ctypes.c_size_t,
                                       ctypes.POINTER(vp)]),
    "ec_upload_wait": (ctypes.c_int, [vp, ctypes.c_size_t]),
    "ec_upload_ready": (ctypes.c_size_t, [vp]),
    "ec_upload_hashes": (ctypes.c_int, [vp, vp]),
    "ec_upload_end": (ctypes.c_int, [vp]),
    "ec_host_alloc": (vp, [ctypes.c_size_t]),
    "ec_host_free": (None, [vp]),
    "ec_device_alloc": (vp, [ctypes.c_size_t]),
    "ec_device_free": (None, [vp]),
    "ec_copy": (ctypes.c_int, [vp, vp, ctypes.c_size_t]),
    "ec_bw_probe": (ctypes.c_int, [ctypes.c_int, vp, ctypes.c_size_t, vp, ctypes.POINTER(ctypes.c_size_t), vp]),
    "ec_encode_shape_probe": (ctypes.c_int, [vp, vp, ctypes.c_size_t, ctypes.c_size_t, vp, ctypes.c_int, vp]),
    "ec_device_count": (ctypes.c_int, []),
    "ec_set_device": (ctypes.c_int, [ctypes.c_int]),
    "ec_encode_kernel_name": (ctypes.c_char_p, [vp]),
    "ec_prepare_encoder": (ctypes.c_int, [vp, ctypes.c_int]),
    "ec_set_body": (ctypes.c_int, [vp, ctypes.c_int]),
    "ec_last_body": (ctypes.c_int, [vp]),
    "ec_encoder_queue_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_ulonglong),
                                              ctypes.POINTER(ctypes.c_ulonglong)]),
    "ec_build_id": (ctypes.c_char_p, []),
}

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def load(path: str = LIB_PATH, partial: bool = False):
    """Load libuplink_ec.so; raises if it is absent (no silent fallback).
    partial: an older build for an A/B (tools/exp, bench.py --lib) may lack
    later exports; those are left unbound instead of failing the load."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process.  PyTorch ships its own libamdhip64.so with
    # the same soname (libamdhip64.so.7) as /opt/rocm's; when torch is loaded
    # first this library binds to that copy.  Loaded the other way round, the
    # process ends up with two runtimes and, once ours has made a HIP call,
    # torch.cuda.is_available() returns False.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if partial and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def strerror(code: int) -> str:
    return load().ec_strerror(code).decode()
