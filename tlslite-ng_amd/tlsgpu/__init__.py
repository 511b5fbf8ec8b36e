"""tlsgpu -- MI355X-native TLS record-layer AEAD engine.

Drop-in for tlslite-ng's bulk-cipher path (tlslite/utils/cipherfactory.py
createAESGCM / createAESCCM / createAESCCM_8 / createCHACHA20 and the AEAD
objects they return), with
hand-written HIP kernels for gfx950 behind a C ABI (include/tlsgpu.h,
libtlsgpu.so) called through ctypes.
"""
from ._lib import TlsGpuError, device_count, get_option, load, options, scratch_info, scratch_trim, helper_info, set_option  # noqa: F401
from .aead import HipAESCCM, HipAESGCM, HipCHACHA20_POLY1305  # noqa: F401
from .batch import KeyTable, make_batch, make_nonces, open_batch, seal_batch  # noqa: F401
from .cipherfactory import (CIPHER_IMPLEMENTATIONS, createAESCCM, createAESCCM_8,  # noqa: F401
                            createAESGCM, createCHACHA20)
from .records import TLS12, TLS13, open_records, seal_records  # noqa: F401
from . import keysetup  # noqa: F401
from .ingest import RecordReader, RecordWriter  # noqa: F401

__version__ = "0.1.0"
