"""ctypes binding of ``libsdfs_cdc.so`` (the C-ABI declared in ``include/sdfs_cdc.h``).

The product path has no CPU fallback: if the HIP library is missing this module raises at import
of the engine (``load()``), and every C-ABI error surfaces as :class:`SdfsCdcError` (the Python
analogue of the ``IOException`` that ``getChunks`` throws in the reference,
SparseDedupFile.java:578-580).
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SDFS_CDC_LIB selects the in-tree measurement build (libsdfs_cdc_tuning.so: kernel-variant
# sweeps and A/B switches, scripts/sweep_scan.py); the default is the product library
DEFAULT_LIB = os.path.join(HERE, "libsdfs_cdc.so")
TUNING_LIB = os.path.join(HERE, "libsdfs_cdc_tuning.so")
LIB_PATH = os.environ.get("SDFS_CDC_LIB") or DEFAULT_LIB
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "sdfs_cdc.h")
HEADER_PATHS = [HEADER_PATH] + [os.path.join(os.path.dirname(HERE), "include", h)
                               for h in ("sdfs_index.h", "sdfs_lz4.h", "sdfs_meta.h", "sdfs_aes.h")]

OK, EINVAL, ECAP, EHIP, ENOMEM, ENODEV = 0, -1, -2, -3, -4, -5
FLAG_DIRECT = 1  # SDFS_CDC_FLAG_DIRECT: no coalescing of concurrent getChunks/getHash calls
SHA256, SHA256_160, MD5 = 0, 1, 2
MIN_GT, MIN_GE = 0, 1
PRED_MASK, PRED_DIV = 0, 1  # sdfs_cdc_params.pred_kind: (fp & mask) == value / fp % div == rem
RECORD_BYTES = 48
NO_STREAM = (1 << 64) - 1  # SDFS_CDC_NO_STREAM
ALL_DEVICES = -1           # sdfs_cdc_params.device: every gfx950 device
FILL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32)


class SdfsCdcError(IOError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"sdfs_cdc error {code}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    """``sdfs_cdc_params`` (include/sdfs_cdc.h)."""

    _fields_ = [
        ("poly", ctypes.c_uint64),
        ("window", ctypes.c_uint32),
        ("min_len", ctypes.c_uint32),
        ("max_len", ctypes.c_uint32),
        ("chunk_length", ctypes.c_uint32),
        ("pred_mask", ctypes.c_uint64),
        ("pred_value", ctypes.c_uint64),
        ("min_cmp", ctypes.c_uint32),
        ("hash_algo", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("max_batch_bytes", ctypes.c_uint64),
        ("device_mask", ctypes.c_uint64),
        ("pred_kind", ctypes.c_uint32),  # ABI 3: boundary detector form
        ("reserved2", ctypes.c_uint32),
        ("pred_div", ctypes.c_uint64),
        ("pred_rem", ctypes.c_uint64),
    ]


class DevOut(ctypes.Structure):
    """``sdfs_cdc_dev_out``: device pointers for the device-resident path."""

    _fields_ = [
        ("counts", ctypes.c_void_p),
        ("starts", ctypes.c_void_p),
        ("lens", ctypes.c_void_p),
        ("digests", ctypes.c_void_p),
        ("cap", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("records", ctypes.c_void_p),
        ("records_cap", ctypes.c_uint64),
        ("total", ctypes.c_void_p),
    ]


# (name, restype, argtypes) for every entry point of include/sdfs_cdc.h
_P = ctypes.POINTER
_u8p, _u32p, _u64p, _vp = _P(ctypes.c_uint8), _P(ctypes.c_uint32), _P(ctypes.c_uint64), ctypes.c_void_p
SIGNATURES = {
    "sdfs_cdc_abi_version": (ctypes.c_int, []),
    "sdfs_cdc_params_default": (ctypes.c_int, [_P(Params), ctypes.c_int]),
    "sdfs_cdc_create": (ctypes.c_int, [_P(Params), _P(_vp)]),
    "sdfs_cdc_destroy": (ctypes.c_int, [_vp]),
    "sdfs_cdc_last_error": (ctypes.c_char_p, []),
    "sdfs_cdc_is_variable_length": (ctypes.c_int, [_vp]),
    "sdfs_cdc_get_max_len": (ctypes.c_int, [_vp]),
    "sdfs_cdc_get_min_len": (ctypes.c_int, [_vp]),
    "sdfs_cdc_set_seed": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sdfs_cdc_digest_len": (ctypes.c_int, [_vp]),
    "sdfs_cdc_slot_cap": (ctypes.c_uint32, [_vp, ctypes.c_uint64]),
    "sdfs_cdc_get_hash": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp]),
    "sdfs_cdc_get_chunks": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_uint32, _u32p]),
    "sdfs_cdc_get_chunks_stream": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp, _vp, _vp,
                                                  ctypes.c_uint32, _u32p]),
    "sdfs_cdc_get_chunks_fill": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32, FILL_FN, _vp, _vp, _vp, _vp,
                                                ctypes.c_uint32, _u32p]),
    "sdfs_cdc_device_count": (ctypes.c_int, [_vp]),
    "sdfs_cdc_device_ordinal": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sdfs_cdc_share_count": (ctypes.c_int, [_vp]),
    "sdfs_cdc_kernel_times_on": (ctypes.c_int, [_vp, ctypes.c_int, _P(ctypes.c_char_p), _P(ctypes.c_float),
                                                ctypes.c_int]),
    "sdfs_cdc_allgather_records": (ctypes.c_int, [_vp, _P(_vp), _u64p, _P(_vp), _P(_vp), ctypes.c_uint64, _u32p,
                                                  _u64p, _P(_vp)]),
    "sdfs_cdc_get_chunks_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp,
                                                 ctypes.c_uint32]),
    "sdfs_cdc_run_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                           _P(DevOut), _vp]),
    "sdfs_cdc_run_device_ragged": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32,
                                                  ctypes.c_uint64, _P(DevOut), _vp]),
    "sdfs_cdc_stream_sync": (ctypes.c_int, [_vp]),
    "sdfs_cdc_queue_stats": (ctypes.c_int, [_vp, _u64p, _u64p]),
    "sdfs_cdc_queue_early": (ctypes.c_int, [_vp, _u64p]),
    "sdfs_cdc_queue_timing": (ctypes.c_int, [_vp, _P(ctypes.c_double), _P(ctypes.c_double), _P(ctypes.c_double)]),
    "sdfs_cdc_set_timing": (ctypes.c_int, [_vp, ctypes.c_int]),
    "sdfs_cdc_set_timing_mask": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_uint32]),
    "sdfs_cdc_kernel_times": (ctypes.c_int, [_vp, _P(ctypes.c_char_p), _P(ctypes.c_float), ctypes.c_int]),
    "sdfs_cdc_synth_device": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, _vp]),
    "sdfs_cdc_host_register": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "sdfs_cdc_host_unregister": (ctypes.c_int, [_vp]),
    "sdfs_cdc_get_hash_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "sdfs_cdc_hash_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    # include/sdfs_index.h
    "sdfs_cdc_index_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, _P(_vp)]),
    "sdfs_cdc_index_destroy": (ctypes.c_int, [_vp]),
    "sdfs_cdc_index_put_records": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp, _vp, _vp,
                                                  _vp, _vp]),
    "sdfs_cdc_index_get": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "sdfs_cdc_index_size": (ctypes.c_int, [_vp, _u64p, _u64p]),
    "sdfs_cdc_index_clear": (ctypes.c_int, [_vp, _vp]),
    "sdfs_cdc_index_set_epoch": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    # include/sdfs_lz4.h
    "sdfs_cdc_lz4_bound": (ctypes.c_uint64, [ctypes.c_uint64]),
    "sdfs_cdc_lz4_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P(_vp)]),
    "sdfs_cdc_lz4_destroy": (ctypes.c_int, [_vp]),
    "sdfs_cdc_lz4_compress_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp,
                                                    ctypes.c_int, _vp]),
    "sdfs_cdc_lz4_plan_records": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint32, _vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "sdfs_cdc_lz4_compress": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _u32p]),
    "sdfs_cdc_lz4_compress_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp,
                                                   ctypes.c_int]),
    "sdfs_cdc_lz4_decompress_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, _vp,
                                                      ctypes.c_int, _vp]),
    "sdfs_cdc_lz4_decompress": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32]),
    # include/sdfs_meta.h
    "sdfs_cdc_map_slot_bytes": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "sdfs_cdc_map_emit": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, _P(DevOut), ctypes.c_uint32, _vp, _vp, _vp,
                                         ctypes.c_uint32, _vp, _vp, _vp]),
    # include/sdfs_aes.h
    "sdfs_cdc_aes_cbc_bound": (ctypes.c_uint64, [ctypes.c_uint64]),
    "sdfs_cdc_aes_create": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_uint32, _P(_vp)]),
    "sdfs_cdc_aes_destroy": (ctypes.c_int, [_vp]),
    "sdfs_cdc_aes_encrypt_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, ctypes.c_int,
                                                   ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sdfs_cdc_aes_decrypt_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, _vp,
                                                   _vp, _vp]),
    "sdfs_cdc_aes_encrypt": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int32, _vp, _vp,
                                            ctypes.c_uint64, _u64p]),
    "sdfs_cdc_aes_decrypt": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _u64p]),
    "sdfs_cdc_aes_encrypt_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_int32,
                                                  _vp, _vp, _vp, _vp]),
}

_lib = None


def load():
    """Load the in-tree HIP library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make` or __graft_entry__.build()")
        # PyTorch-ROCm ships its own libamdhip64 with the same soname: load it first when it is
        # installed so this library binds to the runtime torch uses (one HIP runtime per process;
        # the other order leaves torch with "No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                if LIB_PATH == DEFAULT_LIB:
                    raise ImportError(f"{LIB_PATH} does not export {name}: rebuild it")
                continue  # an older build selected for an A/B measurement
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int) -> int:
    if rc != OK:
        msg = load().sdfs_cdc_last_error()
        raise SdfsCdcError(rc, msg.decode() if msg else "")
    return rc


def default_params(backup_volume: bool = False) -> Params:
    p = Params()
    check(load().sdfs_cdc_params_default(ctypes.byref(p), 1 if backup_volume else 0))
    return p
