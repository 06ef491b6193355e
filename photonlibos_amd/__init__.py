"""photonlibos_amd -- MI355X-native build of PhotonLibOS's payload-checksum path.

Scope: common/checksum CRC32C over the common/iovector buffers
that rpc/ and fs/ push through it. The product is the C-ABI shared library
photonlibos_amd/lib/libphoton_checksum.so (HIP kernels for gfx950 + the
drop-in host entry points of common/checksum/crc32c.h); this Python package is
the host-side mirror of that interface used by tests and bench.py.
"""
from . import checksum  # noqa: F401
from .checksum import (  # noqa: F401
    CrcError,
    crc32c,
    crc32c_extend,
    crc32c_combine,
    crc32c_combine_series,
    crc32c_series,
    crc32c_trim,
)

__all__ = [
    "checksum",
    "CrcError",
    "crc32c",
    "crc32c_extend",
    "crc32c_combine",
    "crc32c_combine_series",
    "crc32c_series",
    "crc32c_trim",
]
