"""ctypes binding of libsmpq.so (the C-ABI declared in include/smpq.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950) and
loaded AFTER ``import torch`` so that its HIP dependency (SONAME libamdhip64.so.7) binds to the
HIP runtime torch already loaded: one runtime, so torch's stream handles are valid here.
There is no fallback: if the library is missing every GPU entry point raises.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the library; see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsmpq.so")
ABI_VERSION = 7

_lib = None
_lock = threading.Lock()

# status codes (include/smpq.h)
SMPQ_OK = 0
SMPQ_E_INVALID = -1
SMPQ_E_SHAPE = -2
SMPQ_E_BITS = -3
SMPQ_E_RANGE = -4
SMPQ_E_CONSTANT = -5
SMPQ_E_HIP = -6
SMPQ_E_INEXACT = -7

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64

_PROTOS = {
    "smpq_abi_version": (_i, []),
    "smpq_last_error": (ctypes.c_char_p, []),
    "smpq_build_stamp": (ctypes.c_char_p, []),
    "smpq_quantize_channels": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp]),
    "smpq_quantize_channels_host": (_i, [_vp, _i, _i, _vp, _vp]),
    "smpq_quantize_channels_ex": (_i, [_vp, _i, _i, _vp, _vp, _vp, _i, _vp]),
    "smpq_quantize_channels_host_ex": (_i, [_vp, _i, _i, _vp, _vp, _i]),
    "smpq_pack_weights": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "smpq_act_absmax": (_i, [_vp, _i, _i64, _vp, _vp]),
    "smpq_act_quantize": (_i, [_vp, _i, _i64, _vp, _i, _vp, _vp]),
    "smpq_pack_weights_ex": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "smpq_maxpool_quantize": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp]),
    "smpq_conv2d_fwd_ex": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp,
                                _vp, _i, _i, _vp, _vp, _i, _vp]),
    "smpq_conv2d_fwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp,
                             _vp, _i, _i, _vp, _vp, _i, _vp]),
    "smpq_conv2d_fwd_q": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp,
                               _vp, _i, _i, _vp, _vp, _vp, ctypes.c_float, _vp, _vp, ctypes.c_float, _i, _vp]),
    "smpq_conv2d_fwd_q_km": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp,
                                  _vp, _i, _i, _vp, _vp, _vp, ctypes.c_float, _vp, _vp, ctypes.c_float, _i, _vp]),
    "smpq_weights_kmajor": (_i, [_vp, _i, _i, _i, _vp, _vp]),
    "smpq_conv2d_pair_supported": (_i, [_i] * 4),
    "smpq_conv2d_chain_supported": (_i, [_i] * 4),
    "smpq_conv2d_chain_ds_supported": (_i, [_i] * 5),
    "smpq_conv2d_chain_fwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, ctypes.c_float,
                                   _vp, _vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, ctypes.c_float, _vp,
                                   ctypes.c_float, _vp,
                                   _vp, _i, _vp, _vp, _vp, ctypes.c_float, _vp, _vp]),
    "smpq_conv2d_pair_fwd": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, ctypes.c_float, _vp,
                                  ctypes.c_float, _vp, _vp, _i, _vp, _vp, _vp, ctypes.c_float, _vp, _vp]),
    "smpq_maxpool_limbs": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "smpq_image_quantize_s2d": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp]),
    "smpq_pack_weights_s2d": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "smpq_pack_weights_s2d_ex": (_i, [_vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp]),
    "smpq_stem_conv_s2d_q": (_i, [_vp, _vp, _i, _i, _i, _vp, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp,
                                  ctypes.c_float, _vp, _i, _vp]),
    "smpq_stem_pool_supported": (_i, [_i] * 6),
    "smpq_stem_pool_s2d_q": (_i, [_vp, _vp, _i, _i, _i, _vp, _i, _i, _vp, _vp, _i, _vp, ctypes.c_float, _vp, _vp]),
    "smpq_conv2d_num_tile_configs": (_i, []),
    "smpq_conv2d_tile_config": (_i, [_i, _vp, _vp, _vp]),
    "smpq_conv2d_tile_kind": (_i, [_i]),
    "smpq_conv2d_tile_supported": (_i, [_i] * 7),
    "smpq_conv2d_workspace_bytes": (ctypes.c_size_t, [_i] * 10),
    "smpq_debug_mfma_i8": (_i, [_vp, _vp, _vp, _vp]),
    "smpq_softmax_xent": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp]),
    "smpq_kl_rows": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp]),
    "smpq_avgpool_fc": (_i, [_vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp]),
    "smpq_fingerprint_chunk_words": (ctypes.c_longlong, []),
    "smpq_fingerprint": (_i, [_vp, _vp, _i, _vp, _vp, _i, _vp, _vp]),
    "smpq_fingerprint_compare": (_i, [_vp, _vp, _i, _vp, _vp]),
    "smpq_fingerprint_host": (ctypes.c_uint64, [_vp, _i64]),
}


EXPORTED_SYMBOLS = tuple(_PROTOS)


class SmpqError(RuntimeError):
    pass


def load(path=None):
    """Load (once) and return the ctypes library; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("SMPQ_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise SmpqError(
                "libsmpq.so not found at %s: build it with `python -c \"import __graft_entry__ as g; "
                "g.build()\"` (the HIP path has no fallback)" % p)
        lib = ctypes.CDLL(p)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.smpq_abi_version()
        if v != ABI_VERSION:
            raise SmpqError("libsmpq ABI version %d, expected %d" % (v, ABI_VERSION))
        _lib = lib
        return lib


def last_error():
    return load().smpq_last_error().decode(errors="replace")


def check(rc, what):
    if rc != SMPQ_OK:
        raise SmpqError("%s failed (%d): %s" % (what, rc, last_error()))
    return rc


def stream_ptr(device=None):
    """Raw hipStream_t of torch's current stream."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
