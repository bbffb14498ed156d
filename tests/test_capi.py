"""CPU tests of the drop-in boundary: the HIP library loads, exports every entry point that
include/sdfs_cdc.h and include/sdfs_index.h declare, the Python mirror binds them all, and the product path fails loudly
(no CPU fallback) when there is no gfx950 device.  No compute calls without a GPU."""
import ctypes
import os
import re

import pytest

from sdfs_amd import _lib
from sdfs_amd.engine import HashFunctionPool, SdfsConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = "".join(open(h).read() for h in _lib.HEADER_PATHS)
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(sdfs_cdc_\w+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_tuning_library_exports_the_same_abi():
    lib = ctypes.CDLL(_lib.TUNING_LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_product_library_reads_no_tuning_environment():
    """Kernel variants and A/B switches exist only in the tuning library: no SDFS_* variable can
    change the product's kernels (the product library does not even contain their names)."""
    prod = open(_lib.DEFAULT_LIB, "rb").read()
    tuning = open(_lib.TUNING_LIB, "rb").read()
    for name in (b"SDFS_SCAN_VARIANT", b"SDFS_HASH_VARIANT", b"SDFS_SEG_LEN", b"SDFS_HASH_WG_PER_CU",
                 b"SDFS_COPY_THREADS", b"SDFS_LZ4_GTAB", b"SDFS_LZ4_STAGE", b"SDFS_AES_VARIANT"):
        assert name not in prod, name
        assert name in tuning, name


def test_python_binding_covers_header():
    assert set(declared_symbols()) == set(_lib.SIGNATURES)
    _lib.load()  # every signature applied without AttributeError


def test_struct_layouts_match_header():
    # sdfs_cdc_params: 8+4+4+4+4+8+8+4+4+4+4+8+8 = 72 bytes (ABI 2 added device_mask), + 4+4+8+8
    # (ABI 3: pred_kind, reserved2, pred_div, pred_rem) = 96; sdfs_cdc_dev_out: 4 ptrs + 2 u32 +
    # ptr + u64 + ptr
    assert ctypes.sizeof(_lib.Params) == 96
    assert ctypes.sizeof(_lib.DevOut) == 64
    assert _lib.load().sdfs_cdc_abi_version() == 3


def test_default_params_are_the_reference_defaults():
    p = _lib.default_params()
    assert p.poly == 10923124345206883 and p.window == 48  # VariableSha256HashEngine.java:41, HashFunctionPool.java:51
    assert p.min_len == 4095 and p.max_len == 32768 and p.chunk_length == 262144  # Main.java:189, VolumeConfigWriter
    b = _lib.default_params(backup_volume=True)
    assert b.max_len == 131072 and b.chunk_length == 40960 * 1024  # VolumeConfigWriter.java:298-307


def test_no_device_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    p = _lib.default_params()
    h = ctypes.c_void_p()
    rc = _lib.load().sdfs_cdc_create(ctypes.byref(p), ctypes.byref(h))
    assert rc == _lib.ENODEV and not h.value
    with pytest.raises(_lib.SdfsCdcError):
        HashFunctionPool().getHashEngine()


def test_invalid_params_rejected_before_device():
    lib = _lib.load()
    for field, val in [("window", 47), ("poly", 0x1FF), ("max_len", 0), ("hash_algo", 9), ("min_cmp", 5),
                       ("device", -7)]:
        p = _lib.default_params()
        setattr(p, field, val)
        h = ctypes.c_void_p()
        assert lib.sdfs_cdc_create(ctypes.byref(p), ctypes.byref(h)) == _lib.EINVAL, field
        assert lib.sdfs_cdc_last_error()


def test_handles_refused_after_destroy_and_unknown():
    """Every handle-taking call on a pointer that is not a live handle fails with EINVAL (no
    use of freed memory), with or without a device."""
    lib = _lib.load()
    bogus = ctypes.c_void_p(0x1234567)
    assert lib.sdfs_cdc_destroy(bogus) == _lib.EINVAL
    assert lib.sdfs_cdc_device_count(bogus) == _lib.EINVAL
    assert lib.sdfs_cdc_share_count(bogus) == _lib.EINVAL
    assert lib.sdfs_cdc_get_max_len(bogus) == -1
    assert lib.sdfs_cdc_slot_cap(bogus, 262144) == 0
    n = ctypes.c_uint32()
    buf = (ctypes.c_uint8 * 64)()
    out = (ctypes.c_uint32 * 8)()
    assert lib.sdfs_cdc_get_chunks(bogus, buf, 64, out, out, None, 8, ctypes.byref(n)) == _lib.EINVAL
    assert lib.sdfs_cdc_destroy(None) == _lib.OK


def test_product_package_never_touches_the_oracle():
    pkg = os.path.join(ROOT, "sdfs_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", src, re.M), f
                assert "libcdc_ref" not in src and "cdc_oracle" not in src and "cdc_ref.h" not in src, f


def test_volume_config_parsing(tmp_path):
    """Config.parseSDFSConfigFile's chunking knobs (Config.java:145-166)."""
    x = tmp_path / "v-volume-cfg.xml"
    x.write_text('<subsystem-config version="master"><io chunk-size="256" hash-type="VARIABLE_SHA256" '
                 'max-variable-segment-size="32" variable-window-size="48" write-threads="8"/></subsystem-config>')
    c = SdfsConfig.from_volume_xml(str(x))
    assert (c.chunk_length, c.min_len, c.max_len, c.window, c.hash_type) == (262144, 4095, 32768, 48, "VARIABLE_SHA256")
    assert c.hash_length == 32 and c.max_hash_cluster == 64  # HashFunctionPool.java:55-66
    x.write_text('<subsystem-config><io chunk-size="40960" hash-type="VARIABLE_MD5" min-variable-segment-size="2"/>'
                 '</subsystem-config>')
    c = SdfsConfig.from_volume_xml(str(x))
    assert c.min_len == 2047 and c.max_len == 40960 * 1024 and c.hash_length == 16
    assert SdfsConfig(hash_type="VARIABLE_SHA256_160").hash_length == 18  # sic, HashFunctionPool.java:58-59
