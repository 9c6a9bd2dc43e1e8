"""ctypes binding of the native ingest engine (``rcdc_ingest_*`` in
include/rcdc.h, ``csrc/rcdc_ingest.cpp``): files -> pack files + pack ids in
host memory, with no Python in the data path (the engine's own threads run
the device pipeline and the host hashing).

Reference: ``FileArchiver::backup_reader`` (archiver/file_archiver.rs:144-160)
and the ``Packer`` (blob/packer.rs: add :304-315, PackSizer :65-200,
add_raw :615-655, save :693-735, finalize :385-398, the pack id
``hash_reader`` :826-836).  This module only marshals: one engine, files
added as bytes or read from a path into the engine's page-locked slots,
callbacks collected into Python lists.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, List, Optional

import numpy as np

from . import _lib
from .errors import status_error

u8, u32, u64 = ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64


class IngestConfig(ctypes.Structure):
    _fields_ = [("key", u8 * 64), ("zstd_level", ctypes.c_int32), ("compress", u32),
                ("extra_verify", u32), ("hash_threads", u32), ("pack_size", u64),
                ("pack_grow_factor", u64), ("pack_size_limit", u64),
                ("pack_current_size", u64), ("batch_bytes", u64), ("depth", u32),
                ("in_slots", u32), ("out_slots", u32), ("pad", u32), ("long_chunk", u64)]


class IngestBlob(ctypes.Structure):
    _fields_ = [("id", u8 * 32), ("offset", u32), ("length", u32),
                ("uncompressed_length", u32), ("type", u32)]


class IngestPack(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("size", u64), ("seq", u64), ("id", u8 * 32),
                ("nblobs", u32), ("header_len", u32), ("blobs", ctypes.POINTER(IngestBlob))]


class IngestFile(ctypes.Structure):
    _fields_ = [("tag", u64), ("len", u64), ("nchunks", u32), ("nnew", u32),
                ("cuts", ctypes.POINTER(u64)), ("ids", ctypes.POINTER(u8))]


class IngestStats(ctypes.Structure):
    _fields_ = [("bytes_in", u64), ("files", u64), ("chunks", u64), ("new_blobs", u64),
                ("packs", u64), ("pack_bytes", u64), ("batches", u64),
                ("seconds", ctypes.c_double)]


assert ctypes.sizeof(IngestBlob) == 48


PACK_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(IngestPack))
FILE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(IngestFile))


def default_config() -> IngestConfig:
    c = IngestConfig()
    _lib.lib().rcdc_ingest_config_default(ctypes.byref(c))
    return c


class NativeIngest:
    """One backup's engine.  ``level``: zstd level (None: a version-1
    repository, blobs stored); ``keep_packs``: copy every pack file into
    ``packs`` (tests; the callback's bytes are only valid during the call).
    Other keyword arguments set ``IngestConfig`` fields."""

    def __init__(self, ctx, key: bytes, level: Optional[int] = 0, extra_verify: bool = True,
                 keep_packs: bool = True, **cfg):
        c = default_config()
        c.key[:] = list(bytes(key))
        c.compress = 0 if level is None else 1
        c.zstd_level = 0 if level is None else int(level)
        c.extra_verify = 1 if extra_verify else 0
        for k, v in cfg.items():
            setattr(c, k, v)
        self.cfg = c
        self.keep_packs = keep_packs
        self.packs: List[dict] = []
        self.files: Dict[int, tuple] = {}
        self._mu = threading.Lock()
        self._pack_cb = PACK_FN(self._on_pack)
        self._file_cb = FILE_FN(self._on_file)
        h = ctypes.c_void_p()
        st = _lib.lib().rcdc_ingest_create(ctx.handle, ctypes.byref(c), self._pack_cb,
                                           self._file_cb, None, ctypes.byref(h))
        if st:
            raise status_error(st, _lib.last_error())
        self._h = h

    # ---- callbacks (engine threads) -----------------------------------------
    def _on_pack(self, _user, pp):
        p = pp.contents
        blobs = [(bytes(b.id), int(b.offset), int(b.length), int(b.uncompressed_length),
                  int(b.type)) for b in p.blobs[:p.nblobs]]
        data = ctypes.string_at(p.data, p.size) if self.keep_packs else None
        with self._mu:
            self.packs.append({"seq": int(p.seq), "size": int(p.size), "id": bytes(p.id),
                               "header_len": int(p.header_len), "blobs": blobs, "data": data})

    def _on_file(self, _user, fp):
        f = fp.contents
        n = int(f.nchunks)
        cuts = np.ctypeslib.as_array(f.cuts, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
        ids = np.ctypeslib.as_array(f.ids, shape=(32 * n,)).reshape(n, 32).copy() if n else \
            np.zeros((0, 32), np.uint8)
        with self._mu:
            self.files[int(f.tag)] = (cuts, ids, int(f.nnew), int(f.len))

    # ---- input ----------------------------------------------------------------
    def _check(self, st):
        if st:
            raise status_error(st, _lib.last_error())

    def add_index(self, ids) -> None:
        a = np.ascontiguousarray(ids, np.uint8).reshape(-1, 32)
        self._check(_lib.lib().rcdc_ingest_add_index(self._h, a.ctypes.data, len(a)))

    def add(self, tag: int, data) -> None:
        a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if isinstance(
            data, (bytes, bytearray, memoryview)) else data, np.uint8)
        self._check(_lib.lib().rcdc_ingest_add(self._h, int(tag), a.ctypes.data if a.size else None,
                                               a.size))

    def add_file(self, tag: int, path: str) -> None:
        """Reserve the file's size, read it straight into the page-locked slot
        (readinto: no intermediate copy), commit what was read."""
        n = os.path.getsize(path)
        buf, ticket = ctypes.c_void_p(), u64()
        self._check(_lib.lib().rcdc_ingest_reserve(self._h, n, ctypes.byref(buf),
                                                   ctypes.byref(ticket)))
        got = 0
        if n:
            mv = memoryview((ctypes.c_char * n).from_address(buf.value)).cast("B")
            with open(path, "rb", buffering=0) as f:
                while got < n:
                    r = f.readinto(mv[got:])
                    if not r:
                        break
                    got += r
        self._check(_lib.lib().rcdc_ingest_commit(self._h, ticket.value, int(tag), got))

    def flush(self) -> None:
        self._check(_lib.lib().rcdc_ingest_flush(self._h))

    def finish(self) -> dict:
        s = IngestStats()
        self._check(_lib.lib().rcdc_ingest_finish(self._h, ctypes.byref(s)))
        self.packs.sort(key=lambda p: p["seq"])
        return {k: getattr(s, k) for k, _ in IngestStats._fields_}

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().rcdc_ingest_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


def sha256_host_one(data) -> bytes:
    """rcdc_sha256_host_one: SHA-256 on the SHA extensions (or scalar)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8))
    out = (u8 * 32)()
    st = _lib.lib().rcdc_sha256_host_one(a.ctypes.data if a.size else None, a.size, out)
    if st:
        raise status_error(st, _lib.last_error())
    return bytes(out)


def sha256_host_ni(bufs, ways: int = 2) -> list:
    """rcdc_sha256_host_ni: SHA-256 of several host buffers, `ways` of them
    interleaved on the SHA extensions of the calling thread."""
    arrs = [np.ascontiguousarray(np.frombuffer(b, np.uint8)) for b in bufs]  # no copy
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrs])
    lens = (ctypes.c_uint64 * max(n, 1))(*[a.size for a in arrs])
    out = (u8 * (32 * max(n, 1)))()
    st = _lib.lib().rcdc_sha256_host_ni(ptrs, lens, n, ways, out)
    if st:
        raise status_error(st, _lib.last_error())
    raw = bytes(out)
    return [raw[32 * i:32 * i + 32] for i in range(n)]
