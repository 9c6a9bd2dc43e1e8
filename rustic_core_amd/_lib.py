"""ctypes binding of ``librcdc.so`` (the C ABI declared in ``include/rcdc.h``).

The library is built in-tree by ``__graft_entry__.build()`` /
``rustic_core_amd/csrc/Makefile``.  There is no fallback: if the shared
library is missing or a symbol is absent, loading raises ``RcdcLibraryError``
-- the chunker never silently runs on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librcdc.so")
# A/B builds of the same sources (tools/ab_lib.sh) load from RCDC_LIB instead
if os.environ.get("RCDC_LIB"):
    LIB_PATH = os.path.abspath(os.environ["RCDC_LIB"])
CSRC = os.path.join(_HERE, "csrc")

# Every entry point of include/rcdc.h (checked by tests/test_abi.py).
EXPORTS = (
    "rcdc_abi_version", "rcdc_last_error", "rcdc_check_params", "rcdc_parse_poly",
    "rcdc_ctx_create", "rcdc_ctx_destroy", "rcdc_max_cuts", "rcdc_chunk_batch",
    "rcdc_stream_open", "rcdc_stream_feed", "rcdc_stream_close", "rcdc_plan_create",
    "rcdc_plan_destroy", "rcdc_plan_run", "rcdc_plan_results", "rcdc_plan_device_results",
    "rcdc_plan_get_info", "rcdc_plan_set_timing", "rcdc_plan_kernel_times", "rcdc_fixed_cuts",
    "rcdc_sha256_chunks", "rcdc_plan_hash", "rcdc_plan_digests", "rcdc_plan_device_digests",
    "rcdc_plan_set_pipeline", "rcdc_plan_hash_many", "rcdc_plan_walk_stats",
    "rcdc_plan_finish", "rcdc_stream_queued", "rcdc_stream_batch_bytes",
    "rcdc_aead_seal", "rcdc_aead_open", "rcdc_pack_build",
    "rcdc_zstd_bound", "rcdc_zstd_compress", "rcdc_zstd_tables", "rcdc_zstd_tables_size",
    "rcdc_zstd_check", "rcdc_pack_build_raw", "rcdc_pack_build_raw_multi", "rcdc_copy_ranges",
    "rcdc_sha256_host", "rcdc_host_alloc", "rcdc_host_free", "rcdc_plan_window",
    "rcdc_ingest_config_default", "rcdc_ingest_create", "rcdc_ingest_add_index",
    "rcdc_ingest_reserve", "rcdc_ingest_commit", "rcdc_ingest_add", "rcdc_ingest_flush",
    "rcdc_ingest_finish", "rcdc_ingest_destroy", "rcdc_sha256_host_one",
    "rcdc_sha256_host_ni", "rcdc_ingest_cancel", "rcdc_ingest_stream_open",
    "rcdc_ingest_stream_reserve", "rcdc_ingest_stream_close", "rcdc_ingest_stream_abort",
    "rcdc_ingest_footprint", "rcdc_ingest_mem_live", "rcdc_index_create", "rcdc_index_destroy",
    "rcdc_index_add", "rcdc_index_size", "rcdc_ingest_set_index",
)
ABI_VERSION = 5


class RcdcLibraryError(RuntimeError):
    """librcdc.so could not be loaded (not built, wrong ABI)."""


class Buf(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64)]


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("scanned_bytes", ctypes.c_uint64),
        ("segments", ctypes.c_uint64),
        ("segment_bytes", ctypes.c_uint32),
        ("work_items", ctypes.c_uint32),
        ("scan_blocks", ctypes.c_uint32),
        ("walk_pieces", ctypes.c_uint32),
        ("walk_seg_bytes", ctypes.c_uint32),
        ("pad", ctypes.c_uint32),
    ]


def build(verbose: bool = False) -> str:
    """Compile librcdc.so for gfx950 with hipcc (cross-compiles without a GPU)."""
    out = subprocess.run(["make", "-s", "-j8", "-C", CSRC], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise RcdcLibraryError(f"building librcdc.so failed:\n{out.stdout}\n{out.stderr}")
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, but NEEDED as "libamdhip64.so").  Loading torch first
    # makes librcdc bind to that already-loaded runtime; loading librcdc
    # first would pull /opt/rocm's copy and torch would then load a second
    # one ("no ROCm-capable device" from whichever initialises last).
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch-free embedding
        pass
    if not os.path.exists(LIB_PATH):
        raise RcdcLibraryError(
            f"{LIB_PATH} not found: build it with __graft_entry__.build() "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - environment specific
        raise RcdcLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name in EXPORTS:
        if not hasattr(L, name):
            raise RcdcLibraryError(f"{LIB_PATH} lacks symbol {name}")
    u64, u32, vp, st = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int
    P = ctypes.POINTER
    L.rcdc_abi_version.restype = u32
    L.rcdc_abi_version.argtypes = []
    if L.rcdc_abi_version() != ABI_VERSION:
        raise RcdcLibraryError("librcdc.so ABI version mismatch")
    L.rcdc_last_error.restype = ctypes.c_char_p
    L.rcdc_last_error.argtypes = []
    L.rcdc_check_params.restype = st
    L.rcdc_check_params.argtypes = [u64, u64, u64]
    L.rcdc_parse_poly.restype = st
    L.rcdc_parse_poly.argtypes = [ctypes.c_char_p, P(u64)]
    L.rcdc_ctx_create.restype = st
    L.rcdc_ctx_create.argtypes = [u64, u64, u64, u64, ctypes.c_int, P(vp)]
    L.rcdc_ctx_destroy.restype = None
    L.rcdc_ctx_destroy.argtypes = [vp]
    L.rcdc_max_cuts.restype = u64
    L.rcdc_max_cuts.argtypes = [vp, u64]
    L.rcdc_chunk_batch.restype = st
    L.rcdc_chunk_batch.argtypes = [vp, P(Buf), u32, vp, u64, vp]
    L.rcdc_stream_open.restype = st
    L.rcdc_stream_open.argtypes = [vp, P(vp)]
    L.rcdc_stream_feed.restype = st
    L.rcdc_stream_feed.argtypes = [vp, vp, u64, ctypes.c_int, vp, u64, P(u64)]
    L.rcdc_stream_queued.restype = u64
    L.rcdc_stream_queued.argtypes = [vp]
    L.rcdc_stream_batch_bytes.restype = u64
    L.rcdc_stream_batch_bytes.argtypes = [vp]
    L.rcdc_plan_finish.restype = st
    L.rcdc_plan_finish.argtypes = [vp]
    L.rcdc_stream_close.restype = None
    L.rcdc_stream_close.argtypes = [vp]
    L.rcdc_plan_create.restype = st
    L.rcdc_plan_create.argtypes = [vp, vp, vp, u32, u64, P(vp)]
    L.rcdc_plan_destroy.restype = None
    L.rcdc_plan_destroy.argtypes = [vp]
    L.rcdc_plan_run.restype = st
    L.rcdc_plan_run.argtypes = [vp, vp, vp]
    L.rcdc_plan_results.restype = st
    L.rcdc_plan_results.argtypes = [vp, vp, u64, vp]
    L.rcdc_plan_device_results.restype = st
    L.rcdc_plan_device_results.argtypes = [vp, P(u64), P(u64), P(P(u64))]
    L.rcdc_plan_get_info.restype = st
    L.rcdc_plan_get_info.argtypes = [vp, P(PlanInfo)]
    L.rcdc_plan_set_timing.restype = st
    L.rcdc_plan_set_timing.argtypes = [vp, ctypes.c_int]
    L.rcdc_plan_kernel_times.restype = st
    L.rcdc_plan_kernel_times.argtypes = [vp, P(u64), P(ctypes.c_double), P(ctypes.c_double)]
    L.rcdc_fixed_cuts.restype = u64
    L.rcdc_fixed_cuts.argtypes = [u64, u64, vp, u64]
    L.rcdc_sha256_chunks.restype = st
    L.rcdc_sha256_chunks.argtypes = [vp, vp, vp, u32, vp, vp]
    L.rcdc_plan_hash.restype = st
    L.rcdc_plan_hash.argtypes = [vp, vp, vp]
    L.rcdc_plan_digests.restype = st
    L.rcdc_plan_digests.argtypes = [vp, vp, u64, vp]
    L.rcdc_plan_hash_many.restype = st
    L.rcdc_plan_hash_many.argtypes = [vp, u32, vp, vp]
    L.rcdc_plan_set_pipeline.restype = st
    L.rcdc_plan_set_pipeline.argtypes = [vp, ctypes.c_int]
    L.rcdc_plan_walk_stats.restype = st
    L.rcdc_plan_walk_stats.argtypes = [vp, vp, vp, u64]
    L.rcdc_aead_seal.restype = st
    L.rcdc_aead_seal.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.rcdc_aead_open.restype = st
    L.rcdc_aead_open.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp]
    L.rcdc_pack_build.restype = st
    L.rcdc_pack_build.argtypes = [vp, vp, vp, vp, u32, vp, u32, vp, u64, vp, vp]
    L.rcdc_pack_build_raw.restype = st
    L.rcdc_pack_build_raw.argtypes = [vp, vp, vp, vp, u32, vp, u32, vp, u64, vp, vp]
    L.rcdc_pack_build_raw_multi.restype = st
    L.rcdc_pack_build_raw_multi.argtypes = [vp, vp, vp, u32, vp, u32, vp, u32, vp, u64, vp, vp]
    L.rcdc_copy_ranges.restype = st
    L.rcdc_copy_ranges.argtypes = [vp, vp, u32, vp, u32, vp, vp]
    L.rcdc_sha256_host.restype = st
    L.rcdc_sha256_host.argtypes = [vp, vp, u32, vp]
    L.rcdc_host_alloc.restype = st
    L.rcdc_host_alloc.argtypes = [u64, vp]
    L.rcdc_host_free.restype = None
    L.rcdc_host_free.argtypes = [vp]
    L.rcdc_zstd_bound.restype = u64
    L.rcdc_zstd_bound.argtypes = [u64]
    L.rcdc_zstd_compress.restype = st
    L.rcdc_zstd_compress.argtypes = [vp, ctypes.c_int, vp, vp, u32, vp, vp, vp]
    L.rcdc_zstd_check.restype = st
    L.rcdc_zstd_check.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp]
    L.rcdc_zstd_tables.restype = None
    L.rcdc_zstd_tables.argtypes = [vp]
    L.rcdc_zstd_tables_size.restype = u64
    L.rcdc_zstd_tables_size.argtypes = []
    L.rcdc_ingest_config_default.restype = None
    L.rcdc_ingest_config_default.argtypes = [vp]
    L.rcdc_ingest_create.restype = st
    L.rcdc_ingest_create.argtypes = [vp, vp, vp, vp, vp, P(vp)]
    L.rcdc_ingest_add_index.restype = st
    L.rcdc_ingest_add_index.argtypes = [vp, vp, u64]
    L.rcdc_ingest_reserve.restype = st
    L.rcdc_ingest_reserve.argtypes = [vp, u64, P(vp), P(u64)]
    L.rcdc_ingest_commit.restype = st
    L.rcdc_ingest_commit.argtypes = [vp, u64, u64, u64]
    L.rcdc_ingest_add.restype = st
    L.rcdc_ingest_add.argtypes = [vp, u64, vp, u64]
    L.rcdc_ingest_flush.restype = st
    L.rcdc_ingest_flush.argtypes = [vp]
    L.rcdc_ingest_finish.restype = st
    L.rcdc_ingest_finish.argtypes = [vp, vp]
    L.rcdc_ingest_destroy.restype = None
    L.rcdc_ingest_destroy.argtypes = [vp]
    L.rcdc_sha256_host_one.restype = st
    L.rcdc_sha256_host_one.argtypes = [vp, u64, vp]
    L.rcdc_sha256_host_ni.restype = st
    L.rcdc_sha256_host_ni.argtypes = [vp, vp, u32, u32, vp]
    L.rcdc_ingest_cancel.restype = st
    L.rcdc_ingest_cancel.argtypes = [vp, u64]
    L.rcdc_ingest_stream_open.restype = st
    L.rcdc_ingest_stream_open.argtypes = [vp, u64, u64, P(u64)]
    L.rcdc_ingest_stream_reserve.restype = st
    L.rcdc_ingest_stream_reserve.argtypes = [vp, u64, u64, P(vp), P(u64)]
    L.rcdc_ingest_stream_close.restype = st
    L.rcdc_ingest_stream_close.argtypes = [vp, u64]
    L.rcdc_ingest_stream_abort.restype = st
    L.rcdc_ingest_stream_abort.argtypes = [vp, u64]
    L.rcdc_ingest_footprint.restype = st
    L.rcdc_ingest_footprint.argtypes = [vp, vp, P(u64), P(u64)]
    L.rcdc_ingest_mem_live.restype = None
    L.rcdc_ingest_mem_live.argtypes = [P(u64), P(u64)]
    L.rcdc_index_create.restype = st
    L.rcdc_index_create.argtypes = [P(vp)]
    L.rcdc_index_destroy.restype = None
    L.rcdc_index_destroy.argtypes = [vp]
    L.rcdc_index_add.restype = st
    L.rcdc_index_add.argtypes = [vp, vp, u64]
    L.rcdc_index_size.restype = u64
    L.rcdc_index_size.argtypes = [vp]
    L.rcdc_ingest_set_index.restype = st
    L.rcdc_ingest_set_index.argtypes = [vp, vp]
    L.rcdc_plan_window.restype = st
    L.rcdc_plan_window.argtypes = [vp, u32, u64, u32, vp, vp]
    L.rcdc_plan_device_digests.restype = st
    L.rcdc_plan_device_digests.argtypes = [vp, P(u64)]
    _lib = L
    return L


def last_error() -> str:
    return lib().rcdc_last_error().decode(errors="replace")
