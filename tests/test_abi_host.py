"""CPU: the C ABI library loads and exports every symbol include/rcdc.h
declares, the host-only entry points match the reference's rules, and the
product path fails loudly without a GPU (no CPU fallback)."""
import ctypes
import io
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "rcdc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(rcdc_[a-z_0-9]+)\s*\(", src, flags=re.M))
    return names


def test_header_symbols_exported(rcdc_lib):
    from rustic_core_amd import _lib
    declared = _header_functions()
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(raw, name), name


def test_abi_version(rcdc_lib):
    assert rcdc_lib.rcdc_abi_version() == 5


def test_ingest_config_layout(rcdc_lib):
    """rcdc_ingest_config as ctypes sees it (native_ingest.IngestConfig) ==
    the C struct: the defaults land in the right fields (ABI 5 added
    max_streams, pack_max_age_ms, slot_max_age_ms)."""
    from rustic_core_amd.native_ingest import IngestConfig, default_config
    assert ctypes.sizeof(IngestConfig) == 152
    c = default_config()
    assert (c.zstd_level, c.compress, c.extra_verify, c.hash_threads) == (0, 1, 1, 10)
    assert (c.pack_size, c.pack_grow_factor, c.pack_size_limit) == (32 << 20, 32, 0xFFFFFFFF)
    assert (c.batch_bytes, c.depth, c.in_slots, c.out_slots) == (2 << 30, 4, 4, 4)
    assert (c.max_streams, c.long_chunk) == (16, 2 << 20)
    assert (c.pack_max_age_ms, c.slot_max_age_ms) == (300000, 1000)  # packer.rs:63 MAX_AGE


def test_shared_index_host(rcdc_lib):
    """rcdc_index: the dedup set engines share (no GPU needed)."""
    import hashlib
    from rustic_core_amd.native_ingest import NativeIndex, mem_live
    ids = np.frombuffer(b"".join(hashlib.sha256(bytes([i])).digest() for i in range(100)),
                        np.uint8)
    idx = NativeIndex(ids)
    assert len(idx) == 100
    assert rcdc_lib.rcdc_index_add(idx.handle, ids.ctypes.data, 100) == 0
    assert len(idx) == 100  # a set
    idx.close()
    assert mem_live() == (0, 0)


@pytest.mark.parametrize("avg,mn,mx,status", [
    (1 << 20, 1 << 19, 1 << 23, 0),
    (1 << 20, 1 << 20, 1 << 20, 0),
    ((1 << 20) + 1, 1 << 19, 1 << 23, 1),   # rabin.rs:22 -> Unsupported
    (3 << 19, 1 << 19, 1 << 23, 1),
    (1 << 20, (1 << 20) + 1, 1 << 23, 1),   # rabin.rs:29
    (1 << 20, 1 << 19, (1 << 20) - 1, 1),   # rabin.rs:35
    (1 << 20, 32, 1 << 23, 1),              # min < 64: rabin.rs:150 slices vec[len-64..]
    (4096, 1024, 16384, 1),                 # min < 4096: rabin.rs:124 underflows
    (4096, 4095, 4096, 1),
    (4096, 4096, 4096, 0),
])
def test_check_params(rcdc_lib, oracle_mod, avg, mn, mx, status):
    assert rcdc_lib.rcdc_check_params(avg, mn, mx) == status
    if mn >= 4096:
        assert oracle_mod.check_params(avg, mn, mx) == (status == 0)
    if status == 1 and mn < 4096:
        assert "4096" in __import__("rustic_core_amd")._lib.last_error()


@pytest.mark.parametrize("poly,ok", [((1 << 8) | 0x1D, False), ((1 << 9) | 0x11, True),
                                     ((1 << 20) | 0x9, True), ((1 << 56) | 0x95, True),
                                     ((1 << 57) | 0x1, False)])
def test_ctx_degree_range(rcdc_lib, poly, ok):
    """deg(P) in 9..56 (polynom_shift = deg - 8 > 0, h << 8 fits
    u64).  Out of range: Unsupported before any HIP call; in range the call
    gets past the degree check (and on a GPU-less host fails at device
    enumeration, never with Unsupported)."""
    from rustic_core_amd import _lib
    h = ctypes.c_void_p()
    st = rcdc_lib.rcdc_ctx_create(poly, 4096, 8192, 65536, 0, ctypes.byref(h))
    if ok:
        assert st != 1, _lib.last_error()
        if st == 0:
            rcdc_lib.rcdc_ctx_destroy(h)
    else:
        assert st == 1 and "degree" in _lib.last_error()


@pytest.mark.parametrize("text,value", [
    ("3da3358b4dc173", 0x003DA3358B4DC173),
    ("3DA3358B4DC173", 0x003DA3358B4DC173),
    ("003da3358b4dc173", 0x003DA3358B4DC173),
    ("+3da3358b4dc173", 0x003DA3358B4DC173),   # from_str_radix accepts '+'
    ("ffffffffffffffff", 0xFFFFFFFFFFFFFFFF),
])
def test_parse_poly_ok(text, value):
    from rustic_core_amd.chunker import ConfigFile
    assert ConfigFile(chunker_polynomial=text).poly() == value


@pytest.mark.parametrize("text", ["", "+", "-1", "0x3da3", "3da3 ", " 3da3", "xyz", "1" * 17])
def test_parse_poly_invalid_input(text):
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.errors import ErrorKind, RusticError
    with pytest.raises(RusticError) as e:
        ConfigFile(chunker_polynomial=text).poly()
    assert e.value.kind == ErrorKind.InvalidInput


def test_config_defaults_and_same_chunker():
    from rustic_core_amd.chunker import Chunker, ConfigFile
    a = ConfigFile.new(2, 0x003DA3358B4DC173)
    assert a.chunker_polynomial == "3da3358b4dc173"
    assert a.get_chunker() is Chunker.Rabin
    assert (a.chunk_size(), a.chunk_min_size(), a.chunk_max_size()) == (1 << 20, 1 << 19, 1 << 23)
    b = ConfigFile.new(2, 0x003DA3358B4DC173)
    assert a.has_same_chunker(b)
    b.chunk_size_ = 1 << 21
    assert not a.has_same_chunker(b)


@pytest.mark.parametrize("n,size", [(0, 1 << 20), (1, 1 << 20), (1 << 20, 1 << 20),
                                    ((1 << 20) + 1, 1 << 20), (33554432, 1045504)])
def test_fixed_cuts_match_oracle(rcdc_lib, oracle_mod, n, size):
    from rustic_core_amd.chunker import fixed_cuts
    assert np.array_equal(fixed_cuts(n, size), oracle_mod.fixed_cuts(n, size))


def test_fixed_size_iter_snapshot(oracle_mod):
    """FixedSizeChunkIter over a reader reproduces fixed_size.rs:82-102."""
    import hashlib
    import json
    from rustic_core_amd.chunker import Chunker, ChunkIter, ConfigFile
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_snapshots.json")))
    data = oracle_mod.stdrng_bytes(23, 32 << 20).tobytes()
    for entry in gold["fixed_chunk_random"]:
        cfg = ConfigFile(chunker=Chunker.FixedSize, chunk_size_=entry["chunk_size"])
        got = [[len(c), hashlib.sha256(c).hexdigest()]
               for c in ChunkIter.from_config(cfg, io.BytesIO(data), len(data))]
        assert got == entry["chunks"]


def test_rabin_path_fails_loudly_without_gpu():
    """No silent CPU fallback: without a device the Rabin iterator raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from rustic_core_amd.chunker import ChunkIter, ConfigFile
    cfg = ConfigFile.new(2, 0x003DA3358B4DC173)
    with pytest.raises(Exception) as e:
        list(ChunkIter.from_config(cfg, io.BytesIO(b"\0" * (1 << 20)), 1 << 20))
    assert "oracle" not in repr(e.value).lower()


def test_product_does_not_import_oracle():
    """The shipped package never routes through the oracle."""
    pkg = os.path.join(ROOT, "rustic_core_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f), errors="replace").read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", text, flags=re.M), f
                assert "cdc_ref" not in text, f


def test_blob_id_entry_points_reject_null(rcdc_lib):
    """rcdc_sha256_chunks / rcdc_plan_hash / rcdc_plan_hash_many /
    rcdc_plan_digests / rcdc_plan_set_pipeline: invalid handles give
    RCDC_ERR_INVALID_INPUT (2, ErrorKind::InvalidInput) before any HIP call;
    more than 8 plans per rcdc_plan_hash_many is rejected the same way."""
    from rustic_core_amd import _lib
    L = _lib.lib()
    assert L.rcdc_sha256_chunks(None, None, None, 1, None, None) == 2
    assert L.rcdc_plan_hash(None, None, None) == 2
    assert L.rcdc_plan_digests(None, None, 0, None) == 2
    assert L.rcdc_plan_set_pipeline(None, 1) == 2
    dd = ctypes.c_uint64(0)
    assert L.rcdc_plan_device_digests(None, ctypes.byref(dd)) == 2
    assert L.rcdc_plan_hash_many(None, 0, None, None) == 0  # nothing to do
    assert L.rcdc_plan_hash_many(None, 1, None, None) == 2
    hs = (ctypes.c_void_p * 9)()
    ars = (ctypes.c_void_p * 9)()
    assert L.rcdc_plan_hash_many(ctypes.cast(hs, ctypes.c_void_p), 9,
                                 ctypes.cast(ars, ctypes.c_void_p), None) == 2
    assert "8 plans" in _lib.last_error()


def test_multi_source_entry_points_reject_bad_input(rcdc_lib):
    """rcdc_pack_build_raw_multi / rcdc_copy_ranges (ABI 3): a null context,
    no input buffers or a null source give RCDC_ERR_INVALID_INPUT before any
    HIP call."""
    from rustic_core_amd import _lib
    L = _lib.lib()
    key = (ctypes.c_uint8 * 64)()
    assert L.rcdc_pack_build_raw_multi(None, key, None, 0, None, 0, None, 0, None, 0,
                                       None, None) == 2
    assert "no input buffers" in _lib.last_error()
    srcs = (ctypes.c_void_p * 2)(None, None)
    assert L.rcdc_pack_build_raw_multi(None, key, ctypes.cast(srcs, ctypes.c_void_p), 2, None,
                                       0, None, 0, None, 0, None, None) == 2
    assert "source 0 is null" in _lib.last_error()
    assert L.rcdc_copy_ranges(None, None, 0, None, 0, None, None) == 2
