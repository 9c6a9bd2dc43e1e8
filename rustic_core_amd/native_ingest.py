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
                ("in_slots", u32), ("out_slots", u32), ("max_streams", u32), ("long_chunk", u64),
                ("pack_max_age_ms", u32), ("slot_max_age_ms", u32)]


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
        (readinto: no intermediate copy), commit what was read.  A read that
        fails cancels the reservation (rcdc_ingest_cancel: the reference logs
        and skips the file, archiver.rs:197-203) and re-raises."""
        n = os.path.getsize(path)
        if n > self.cfg.batch_bytes:
            with open(path, "rb", buffering=0) as f:
                self.add_stream(tag, f, size_hint=n)
            return
        buf, ticket = ctypes.c_void_p(), u64()
        self._check(_lib.lib().rcdc_ingest_reserve(self._h, n, ctypes.byref(buf),
                                                   ctypes.byref(ticket)))
        got = 0
        try:
            with open(path, "rb", buffering=0) as f:
                if n:
                    mv = memoryview((ctypes.c_char * n).from_address(buf.value)).cast("B")
                    while got < n:
                        r = f.readinto(mv[got:])
                        if not r:
                            break
                        got += r
                # a file that grew since its size was taken: the reference
                # reads to EOF (rabin.rs:110-191), so this one goes as a stream
                grew = got == n and f.read(1)
                if grew:
                    _lib.lib().rcdc_ingest_cancel(self._h, ticket.value)
                    f.seek(0)
                    self.add_stream(tag, f, size_hint=n)
                    return
        except BaseException:
            _lib.lib().rcdc_ingest_cancel(self._h, ticket.value)
            raise
        self._check(_lib.lib().rcdc_ingest_commit(self._h, ticket.value, int(tag), got))

    # ---- streams: any Read, of any or unknown length ---------------------------
    def stream_open(self, tag: int, size_hint: int = 0) -> int:
        h = u64()
        self._check(_lib.lib().rcdc_ingest_stream_open(self._h, int(tag), int(size_hint),
                                                       ctypes.byref(h)))
        return h.value

    def stream_reserve(self, stream: int, n: int):
        """(memoryview of n page-locked bytes, ticket) for the stream's next piece."""
        buf, ticket = ctypes.c_void_p(), u64()
        self._check(_lib.lib().rcdc_ingest_stream_reserve(self._h, stream, int(n),
                                                          ctypes.byref(buf), ctypes.byref(ticket)))
        mv = memoryview((ctypes.c_char * max(n, 1)).from_address(buf.value)).cast("B")[:n]
        return mv, ticket.value

    def commit(self, ticket: int, n: int, tag: int = 0) -> None:
        self._check(_lib.lib().rcdc_ingest_commit(self._h, ticket, int(tag), int(n)))

    def cancel(self, ticket: int) -> None:
        self._check(_lib.lib().rcdc_ingest_cancel(self._h, ticket))

    def stream_close(self, stream: int) -> None:
        self._check(_lib.lib().rcdc_ingest_stream_close(self._h, stream))

    def stream_abort(self, stream: int) -> None:
        self._check(_lib.lib().rcdc_ingest_stream_abort(self._h, stream))

    def add_stream(self, tag: int, reader, piece: Optional[int] = None, size_hint: int = 0) -> int:
        """Feed a readable binary object (readinto) until EOF as one file:
        ChunkIter::from_config(cfg, reader, size_hint) (chunker.rs:22-47).  A
        failing read aborts the stream (its completed chunks stay packed, as
        Packer::add had them) and re-raises.  Returns the bytes read.
        piece: bytes per reservation (default 16 MiB, at most a quarter batch,
        as rcdc_ingest_add cuts a large file)."""
        if piece is None:
            piece = max(min(16 << 20, self.cfg.batch_bytes // 4) & ~255, 256)
        h = self.stream_open(tag, size_hint)
        total = 0
        try:
            while True:
                mv, t = self.stream_reserve(h, piece)
                got = 0
                try:
                    while got < piece:
                        r = reader.readinto(mv[got:])
                        if not r:
                            break
                        got += r
                    self.commit(t, got)
                except BaseException:
                    _lib.lib().rcdc_ingest_cancel(self._h, t)  # (a no-op once committed)
                    raise
                total += got
                if got < piece:
                    break
        except BaseException:
            _lib.lib().rcdc_ingest_stream_abort(self._h, h)
            raise
        self.stream_close(h)
        return total

    def set_index(self, index: "NativeIndex") -> None:
        """Dedup against a set shared with other engines (multi-device ingest)."""
        self._check(_lib.lib().rcdc_ingest_set_index(self._h, index.handle))
        self._index = index  # keep it alive while the engine uses it

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


class NativeIndex:
    """rcdc_index: one dedup set shared by the engines of several devices, so
    each blob is packed once per backup (the reference's single Packer,
    archiver.rs:195, blob/packer.rs:304-315)."""

    def __init__(self, ids=None):
        h = ctypes.c_void_p()
        st = _lib.lib().rcdc_index_create(ctypes.byref(h))
        if st:
            raise status_error(st, _lib.last_error())
        self.handle = h
        if ids is not None and len(ids):
            a = np.ascontiguousarray(ids, np.uint8).reshape(-1, 32)
            st = _lib.lib().rcdc_index_add(h, a.ctypes.data, len(a))
            if st:
                raise status_error(st, _lib.last_error())

    def __len__(self) -> int:
        return int(_lib.lib().rcdc_index_size(self.handle))

    def close(self) -> None:
        if getattr(self, "handle", None):
            _lib.lib().rcdc_index_destroy(self.handle)
            self.handle = None


class MultiIngest:
    """N engines (one per device context) behind one file router and one
    dedup set.  Files go to the engine with the fewest bytes so far (greedy
    LPT online; shard.assign_lpt is the same rule offline); every engine
    dedups against the shared NativeIndex, so a chunk found by several
    engines is packed by exactly one.  Results: the union of the engines'
    files and packs."""

    def __init__(self, ctxs, key: bytes, level: Optional[int] = 0, index_ids=None, **cfg):
        self.index = NativeIndex(index_ids)
        self.engines = []
        try:
            for c in ctxs:
                e = NativeIngest(c, key, level=level, **cfg)
                e.set_index(self.index)
                self.engines.append(e)
        except BaseException:
            self.close()
            raise
        self.load = [0] * len(self.engines)
        self._mu = threading.Lock()

    def _pick(self, n: int) -> "NativeIngest":
        with self._mu:
            i = min(range(len(self.load)), key=lambda j: (self.load[j], j))
            self.load[i] += n
        return self.engines[i]

    def add(self, tag: int, data) -> None:
        a = np.frombuffer(bytes(data), np.uint8) if isinstance(
            data, (bytes, bytearray, memoryview)) else np.asarray(data)
        self._pick(int(a.size)).add(tag, a)

    def add_file(self, tag: int, path: str) -> None:
        self._pick(os.path.getsize(path)).add_file(tag, path)

    def finish(self) -> dict:
        """The engines' stats summed (their wall time: the longest)."""
        tot: Dict[str, float] = {}
        for e in self.engines:
            for k, v in e.finish().items():
                tot[k] = max(tot.get(k, 0), v) if k == "seconds" else tot.get(k, 0) + v
        return tot

    @property
    def files(self) -> Dict[int, tuple]:
        out: Dict[int, tuple] = {}
        for e in self.engines:
            out.update(e.files)
        return out

    @property
    def packs(self) -> List[dict]:
        return [p for e in self.engines for p in e.packs]

    def close(self) -> None:
        for e in self.engines:
            e.close()
        self.engines = []
        self.index.close()


def mem_live():
    """(page-locked, device) bytes held by the process's ingest engines."""
    p, d = u64(), u64()
    _lib.lib().rcdc_ingest_mem_live(ctypes.byref(p), ctypes.byref(d))
    return p.value, d.value


def footprint(ctx, **cfg):
    """(page-locked, device) bytes rcdc_ingest_create allocates for cfg."""
    c = default_config()
    for k, v in cfg.items():
        setattr(c, k, v)
    p, d = u64(), u64()
    st = _lib.lib().rcdc_ingest_footprint(ctx.handle, ctypes.byref(c), ctypes.byref(p),
                                          ctypes.byref(d))
    if st:
        raise status_error(st, _lib.last_error())
    return p.value, d.value


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
