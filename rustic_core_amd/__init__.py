"""rustic_core_amd -- MI355X-native content-defined chunker for rustic_core.

Replaces the Rabin CDC hot path of rustic_core (crates/core/src/chunker*)
with hand-written gfx950 HIP kernels behind the C ABI of ``include/rcdc.h``
(``librcdc.so``).  The Python layer mirrors the reference's chunker surface
(``ChunkIter.from_config``, ``check_rabin_params``, ``ConfigFile``) and the
device-resident batch API used by ``bench.py``.
"""
from .errors import ErrorKind, RusticError  # noqa: F401
from .chunker import (  # noqa: F401
    Chunker, ChunkIter, ConfigFile, Context, RabinChunkIter, FixedSizeChunkIter,
    check_rabin_params, fixed_cuts, DEFAULT_CHUNK_SIZE, DEFAULT_CHUNK_MIN_SIZE,
    DEFAULT_CHUNK_MAX_SIZE,
)

__all__ = [
    "ErrorKind", "RusticError", "Chunker", "ChunkIter", "ConfigFile", "Context",
    "RabinChunkIter", "FixedSizeChunkIter", "check_rabin_params", "fixed_cuts",
]
