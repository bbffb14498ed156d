"""sdfs_amd — MI355X-native variable-block CDC + fingerprint engine for SDFS's write path.

The drop-in boundary is the C-ABI in ``include/sdfs_cdc.h`` (``libsdfs_cdc.so``, hand-written
gfx950 HIP kernels); this package is the host-side mirror of the reference's
``org.opendedup.hashing`` plugin surface on top of it.  See DESIGN.md / INTEGRATION.md.
"""
from ._lib import MD5, MIN_GE, MIN_GT, RECORD_BYTES, SHA256, SHA256_160, SdfsCdcError  # noqa: F401
from .engine import (  # noqa: F401
    POLY,
    VARIABLE_MD5,
    VARIABLE_SHA256,
    VARIABLE_SHA256_160,
    Finger,
    HashFunctionPool,
    HipVariableMD5HashEngine,
    HipVariableSha256HashEngine,
    SdfsConfig,
)

__all__ = [
    "Finger", "HashFunctionPool", "HipVariableMD5HashEngine", "HipVariableSha256HashEngine", "SdfsConfig",
    "SdfsCdcError", "POLY", "VARIABLE_MD5", "VARIABLE_SHA256", "VARIABLE_SHA256_160",
]
