"""Host-side mirror of rustic_core's chunker surface, backed by librcdc.

Reference (rustic_core 0.12.0):
  crates/core/src/chunker.rs:16-59          ChunkIter::{Rabin, FixedSize}, from_config
  crates/core/src/chunker/rabin.rs:17-42    check_rabin_params
  crates/core/src/chunker/rabin.rs:82-191   RabinChunkIter::{new, next}
  crates/core/src/chunker/fixed_size.rs     FixedSizeChunkIter
  crates/core/src/repofile/configfile.rs    ConfigFile chunker fields / getters

``ChunkIter.from_config(config, reader, size_hint)`` returns an iterator that
yields every chunk of ``reader`` as ``bytes``, exactly the chunks the Rust
iterator yields.  For Rabin the cut points come from the MI355X kernels
(rcdc_stream_feed); the bytes themselves never leave the host buffer.
There is no CPU fallback for the Rabin path: without librcdc.so or a GPU the
constructor raises.
"""
from __future__ import annotations

import collections
import ctypes
import enum
import io
import os
import threading
from dataclasses import dataclass
from typing import Iterator, Optional

import numpy as np

from . import _lib
from .errors import ErrorKind, RusticError, status_error

KB = 1024
MB = 1024 * KB
# configfile.rs:36-41
DEFAULT_CHUNK_SIZE = 1 * MB
DEFAULT_CHUNK_MIN_SIZE = 512 * KB
DEFAULT_CHUNK_MAX_SIZE = 8 * MB
# Bytes requested from the reader per read(): large reads, the cut points do
# not depend on how the stream is split (the reference reads 4 KiB, rabin.rs:12).
READ_SIZE = int(os.environ.get("RCDC_READ_MIB", "16")) * MB


class Chunker(enum.Enum):
    """configfile.rs `Chunker` (default Rabin)."""
    Rabin = "rabin"
    FixedSize = "fixed_size"


@dataclass
class ConfigFile:
    """The chunker-related fields of rustic's repository ``ConfigFile``."""
    version: int = 2
    chunker_polynomial: str = ""
    chunker: Optional[Chunker] = None
    chunk_size_: Optional[int] = None
    chunk_min_size_: Optional[int] = None
    chunk_max_size_: Optional[int] = None
    # pack sizing (configfile.rs:60-100), used by rustic_core_amd.pack
    treepack_size: Optional[int] = None
    treepack_growfactor: Optional[int] = None
    treepack_size_limit: Optional[int] = None
    datapack_size: Optional[int] = None
    datapack_growfactor: Optional[int] = None
    datapack_size_limit: Optional[int] = None
    min_packsize_tolerate_percent: Optional[int] = None
    max_packsize_tolerate_percent: Optional[int] = None
    # blob processing (configfile.rs:43-50)
    compression: Optional[int] = None
    extra_verify: Optional[bool] = None

    @classmethod
    def new(cls, version: int, poly: int) -> "ConfigFile":
        # configfile.rs:151-158: format!("{poly:x}")
        return cls(version=version, chunker_polynomial=f"{poly:x}")

    def poly(self) -> int:
        """configfile.rs:165-175 (`u64::from_str_radix(.., 16)`)."""
        out = ctypes.c_uint64(0)
        st = _lib.lib().rcdc_parse_poly(self.chunker_polynomial.encode(), ctypes.byref(out))
        if st:
            raise status_error(st, _lib.last_error())
        return out.value

    def packsize(self, blob_type: int):
        """configfile.rs:211-231: (size, grow factor, limit) for BlobType
        0 = data, 1 = tree."""
        MB = 1 << 20
        if blob_type == 1:
            return (4 * MB if self.treepack_size is None else self.treepack_size,
                    32 if self.treepack_growfactor is None else self.treepack_growfactor,
                    0xFFFFFFFF if self.treepack_size_limit is None else self.treepack_size_limit)
        return (32 * MB if self.datapack_size is None else self.datapack_size,
                32 if self.datapack_growfactor is None else self.datapack_growfactor,
                0xFFFFFFFF if self.datapack_size_limit is None else self.datapack_size_limit)

    def packsize_ok_percents(self):
        """configfile.rs:236-245."""
        mx = self.max_packsize_tolerate_percent
        return (30 if self.min_packsize_tolerate_percent is None
                else self.min_packsize_tolerate_percent,
                0xFFFFFFFF if not mx else mx)

    def zstd(self) -> Optional[int]:
        """configfile.rs:182-193: the zstd level, None = no compression."""
        if self.version == 1 or (self.version == 2 and self.compression == 0):
            return None
        if self.version == 2:
            return 0 if self.compression is None else self.compression
        raise RusticError(ErrorKind.Unsupported,
                          f"Config version `{self.version}` not supported. Please make sure, "
                          "that you use the correct version.")

    def extra_verify_(self) -> bool:
        """configfile.rs:197-199 (default: verify)."""
        return True if self.extra_verify is None else bool(self.extra_verify)

    def get_chunker(self) -> Chunker:
        return self.chunker or Chunker.Rabin

    def chunk_size(self) -> int:
        return DEFAULT_CHUNK_SIZE if self.chunk_size_ is None else self.chunk_size_

    def chunk_min_size(self) -> int:
        return DEFAULT_CHUNK_MIN_SIZE if self.chunk_min_size_ is None else self.chunk_min_size_

    def chunk_max_size(self) -> int:
        return DEFAULT_CHUNK_MAX_SIZE if self.chunk_max_size_ is None else self.chunk_max_size_

    def has_same_chunker(self, other: "ConfigFile") -> bool:
        """configfile.rs:274-285."""
        if self.get_chunker() != other.get_chunker():
            return False
        if self.get_chunker() == Chunker.Rabin:
            return (self.chunker_polynomial == other.chunker_polynomial
                    and self.chunk_size() == other.chunk_size()
                    and self.chunk_min_size() == other.chunk_min_size()
                    and self.chunk_max_size() == other.chunk_max_size())
        return self.chunk_size() == other.chunk_size()


def check_rabin_params(chunk_size: int, chunk_min_size: int, chunk_max_size: int) -> None:
    """rabin.rs:17-42 -- raises ``RusticError(ErrorKind.Unsupported)``."""
    st = _lib.lib().rcdc_check_params(chunk_size, chunk_min_size, chunk_max_size)
    if st:
        raise status_error(st, _lib.last_error())


# ---------------------------------------------------------------------------
# device contexts (one per (poly, params, device); the reference rebuilds the
# Rabin64 tables per file at chunker.rs:30, we build them once)
# ---------------------------------------------------------------------------
_ctx_lock = threading.Lock()
_ctx_cache: dict = {}


def default_device() -> int:
    return int(os.environ.get("RCDC_DEVICE", os.environ.get("LOCAL_RANK", "0")))


class Context:
    """Owns an ``rcdc_ctx`` (tables on one device + chunker parameters)."""

    def __init__(self, poly: int, min_size: int, avg: int, max_size: int,
                 device: Optional[int] = None):
        L = _lib.lib()
        self.poly, self.min_size, self.avg, self.max_size = poly, min_size, avg, max_size
        self.device = default_device() if device is None else device
        h = ctypes.c_void_p()
        st = L.rcdc_ctx_create(poly, min_size, avg, max_size, self.device, ctypes.byref(h))
        if st:
            raise status_error(st, _lib.last_error())
        self._h = h

    @classmethod
    def get(cls, poly: int, min_size: int, avg: int, max_size: int,
            device: Optional[int] = None) -> "Context":
        dev = default_device() if device is None else device
        key = (poly, min_size, avg, max_size, dev)
        with _ctx_lock:
            c = _ctx_cache.get(key)
            if c is None:
                c = cls(poly, min_size, avg, max_size, dev)
                _ctx_cache[key] = c
            return c

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def max_cuts(self, n: int) -> int:
        return int(_lib.lib().rcdc_max_cuts(self._h, n))

    def chunk_batch(self, buffers) -> list:
        """Chunk independent host buffers; returns one ``np.uint64`` cut array each."""
        bufs = [np.ascontiguousarray(np.frombuffer(b, dtype=np.uint8)) if not isinstance(
            b, np.ndarray) else np.ascontiguousarray(b, dtype=np.uint8).reshape(-1)
            for b in buffers]
        n = len(bufs)
        arr = (_lib.Buf * max(n, 1))()
        cap = 0
        for i, b in enumerate(bufs):
            arr[i].data = b.ctypes.data if b.size else None
            arr[i].len = b.size
            cap += self.max_cuts(b.size)
        cuts = np.zeros(max(cap, 1), dtype=np.uint64)
        counts = np.zeros(max(n, 1), dtype=np.uint64)
        st = _lib.lib().rcdc_chunk_batch(self._h, arr, n, cuts.ctypes.data, cap,
                                         counts.ctypes.data)
        if st:
            raise status_error(st, _lib.last_error())
        out, o = [], 0
        for i in range(n):
            k = int(counts[i])
            out.append(cuts[o:o + k].copy())
            o += k
        return out

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            if getattr(self, "_h", None):
                _lib.lib().rcdc_ctx_destroy(self._h)
                self._h = None
        except Exception:
            pass


class _Stream:
    """rcdc_stream: one file fed in pieces; returns final cut offsets."""

    def __init__(self, ctx: Context):
        self._ctx = ctx
        h = ctypes.c_void_p()
        st = _lib.lib().rcdc_stream_open(ctx.handle, ctypes.byref(h))
        if st:
            raise status_error(st, _lib.last_error())
        self._h = h

    def feed(self, data, is_final: bool) -> np.ndarray:
        """Feed one piece; returns every cut that became final (the C ABI
        hands out at most `cap` per call and queues the rest: drained here)."""
        L = _lib.lib()
        a = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(0, np.uint8)
        cap = self._ctx.max_cuts(len(a)) + 1
        out = []
        n = ctypes.c_uint64(0)
        first = True
        while True:
            cuts = np.zeros(cap, dtype=np.uint64)
            st = L.rcdc_stream_feed(self._h, a.ctypes.data if (first and a.size) else None,
                                    a.size if first else 0, int(is_final), cuts.ctypes.data,
                                    cap, ctypes.byref(n))
            if st:
                raise status_error(st, _lib.last_error())
            first = False
            out.append(cuts[:n.value])
            q = int(L.rcdc_stream_queued(self._h))
            if q == 0:
                break
            cap = q
        return out[0] if len(out) == 1 else np.concatenate(out)

    def close(self):
        if self._h:
            _lib.lib().rcdc_stream_close(self._h)
            self._h = None

    __del__ = close


def _read(reader, n: int) -> bytes:
    """One reader.read(n) with the reference's error mapping (rabin.rs:162-181)."""
    while True:
        try:
            b = reader.read(n)
        except InterruptedError:
            continue  # ErrorKind::Interrupted -> retry (rabin.rs:173)
        except OSError as e:
            raise RusticError(ErrorKind.InputOutput,
                              f"Failed to read from reader in iterator: {e}") from e
        return b if b is not None else b""


def _read_into(reader, mv: memoryview) -> int:
    """reader.readinto(mv) (no intermediate bytes object) with the same error
    mapping; readers without readinto go through read()."""
    readinto = getattr(reader, "readinto", None)
    while True:
        try:
            if readinto is None:
                raise NotImplementedError
            n = readinto(mv)
        except NotImplementedError:  # e.g. an io.RawIOBase that only has read()
            b = _read(reader, len(mv))
            mv[:len(b)] = b
            return len(b)
        except InterruptedError:
            continue  # ErrorKind::Interrupted -> retry (rabin.rs:173)
        except OSError as e:
            raise RusticError(ErrorKind.InputOutput,
                              f"Failed to read from reader in iterator: {e}") from e
        return n or 0


# Read blocks: READ_SIZE buffers in page-locked memory (rcdc_host_alloc), so
# that rcdc_stream_feed DMAs each read straight to the device instead of
# copying it through its staging slots; reused across iterators (allocation
# costs milliseconds).  A block takes further reads while at least MIN_READ
# bytes of it are free.
_POOL: collections.deque = collections.deque()
# (what concurrent iterators held at once is kept, up to this many blocks)
_POOL_MAX = int(os.environ.get("RCDC_BLOCK_POOL", "32"))
MIN_READ = 1 * MB


class _Block:
    __slots__ = ("ptr", "mv", "addr", "_keep")

    def __init__(self):
        p = ctypes.c_void_p()
        self.ptr = None
        try:
            if _lib.lib().rcdc_host_alloc(READ_SIZE, ctypes.byref(p)) == 0:
                self.ptr = p.value
        except Exception:  # no librcdc: the iterator's constructor raises anyway
            pass
        if self.ptr:
            self._keep = None
            self.mv = memoryview((ctypes.c_char * READ_SIZE).from_address(self.ptr)).cast("B")
        else:  # page-locked memory refused: pageable (the feed stages it)
            self._keep = bytearray(READ_SIZE)
            self.mv = memoryview(self._keep)
        self.addr = ctypes.addressof(ctypes.c_char.from_buffer(self.mv))

    def __del__(self):
        if self.ptr:
            try:
                _lib.lib().rcdc_host_free(self.ptr)
            except Exception:  # interpreter shutdown
                pass
            self.ptr = None


_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = (ctypes.c_void_p, ctypes.c_ssize_t)
_BYTES_DATA = bytes.__basicsize__ - 1  # offset of PyBytesObject.ob_sval


def _block() -> _Block:
    try:
        return _POOL.pop()
    except IndexError:
        return _Block()


def _release(blk: _Block) -> None:
    if len(_POOL) < _POOL_MAX:
        _POOL.append(blk)


# Live iterators: when the last one finishes, the pool keeps only
# _POOL_IDLE blocks, so an idle process holds _POOL_IDLE x READ_SIZE of
# page-locked memory (not _POOL_MAX x READ_SIZE).
_POOL_IDLE = int(os.environ.get("RCDC_BLOCK_POOL_IDLE", "2"))
_live = 0
_live_lock = threading.Lock()


def _iter_started() -> None:
    global _live
    with _live_lock:
        _live += 1


def _iter_done() -> None:
    global _live
    with _live_lock:
        _live -= 1
        if _live == 0:
            while len(_POOL) > _POOL_IDLE:
                try:
                    _POOL.popleft()  # freed by _Block.__del__
                except IndexError:
                    break


# Large files run as a pipeline of three threads: the reader thread reads
# block after block, the feeder thread feeds each read to the device stream
# (rcdc_stream_feed: H2D, chunking, cuts back), and the caller's thread
# copies the chunks out.  All three release the GIL in their native calls, so
# a file's reads, device passes and chunk copies overlap (one-thread order
# was read -> feed -> copies, ~28 ms per 256 MiB, tools/c1_profile.py).
# PIPE_BLOCKS bounds the blocks one iterator holds (read, fed or not yet
# copied out), raised to what the device stream needs to see a cut: it runs
# a pass only once rcdc_stream_batch_bytes are buffered after its last cut,
# and the consumer frees no block until then (with 2 blocks of reads short
# of 16 MiB the pipe waited for itself: tools/soak_stream.py).
PIPE_BLOCKS = int(os.environ.get("RCDC_PIPE_BLOCKS", "4"))


def _pipe_blocks(ctx) -> int:
    """Blocks a pipe may hold: the block with the consumer's position
    (as little as 1 unconsumed byte), enough blocks of >= READ_SIZE -
    MIN_READ bytes to reach the stream's pass size, and the one being read."""
    h = getattr(ctx, "handle", None)
    batch = int(_lib.lib().rcdc_stream_batch_bytes(h)) if h is not None else \
        max(16 * MB, 2 * ctx.max_size + 256)
    need = 2 + -(-batch // (READ_SIZE - MIN_READ))
    return max(PIPE_BLOCKS, need)


class _Pipe:
    """The reader and feeder threads of one iterator.  Items on `out`, in
    file order: (block, start, n, retire_block, cuts, eof), or an exception
    to raise where the consumer reaches it."""

    def __init__(self, reader, stream, first, blocks):
        self.reader, self.stream = reader, stream
        self.stop = threading.Event()
        self.room = threading.Semaphore(blocks - 1)  # (`first`'s block is held)
        self.feed_q = collections.deque()
        self.feed_cv = threading.Condition()
        self.out = collections.deque()
        self.out_cv = threading.Condition()
        self._put_feed(first)
        self.blk, self.pos = (None, 0) if first[3] else (first[0], first[1] + first[2])
        self.t_read = threading.Thread(target=self._read_loop, name="rcdc-read", daemon=True)
        self.t_feed = threading.Thread(target=self._feed_loop, name="rcdc-feed", daemon=True)
        self.t_feed.start()
        self.t_read.start()

    def _put_feed(self, item):
        with self.feed_cv:
            self.feed_q.append(item)
            self.feed_cv.notify()

    def _put_out(self, item):
        with self.out_cv:
            self.out.append(item)
            self.out_cv.notify()

    def _read_loop(self):
        try:
            while not self.stop.is_set():
                if self.blk is None:
                    while not self.room.acquire(timeout=0.05):
                        if self.stop.is_set():
                            return
                    self.blk, self.pos = _block(), 0
                blk, p = self.blk, self.pos
                n = _read_into(self.reader, blk.mv[p:])
                self.pos = p + n
                retire = not n or READ_SIZE - self.pos < MIN_READ
                if retire:
                    self.blk = None
                self._put_feed((blk, p, n, retire))
                if not n:
                    return
        except BaseException as e:  # RusticError (read), or anything else
            self._put_feed(e)
        finally:
            self._put_feed(None)  # the feeder's end

    def _feed_loop(self):
        while True:
            with self.feed_cv:
                while not self.feed_q:
                    self.feed_cv.wait()
                item = self.feed_q.popleft()
            if item is None:
                return
            if isinstance(item, BaseException):
                self._put_out(item)
                return
            blk, p, n, retire = item
            try:
                cuts = self.stream.feed(blk.mv[p:p + n], not n) if not self.stop.is_set() else None
            except BaseException as e:
                self.stop.set()
                self._put_out(e)
                return
            if cuts is None:
                return
            self._put_out((blk, p, n, retire, cuts, not n))
            if not n:
                return

    def get(self):
        with self.out_cv:
            while not self.out:
                self.out_cv.wait()
            return self.out.popleft()

    def close(self):
        """Stop reading and feeding; returns once neither thread can touch a
        block or the stream again."""
        self.stop.set()
        self.t_read.join()
        self.t_feed.join()


class RabinChunkIter:
    """rabin.rs ChunkIter with device-computed cut points.

    Yields ``bytes`` chunks; raises ``RusticError`` like the reference's
    ``Some(Err(..))`` items (after which iteration stops).  The reader fills
    pooled page-locked blocks in place; every read is fed to the device
    stream as it lands; a chunk is one copy out of the block(s) it lies in.
    A file whose first read fills a whole block goes through a _Pipe.
    """

    def __init__(self, ctx: Context, reader, size_hint: int = 0):
        check_rabin_params(ctx.avg, ctx.min_size, ctx.max_size)
        self._ctx = ctx
        self._reader = reader
        self.size_hint = size_hint  # capacity hint only; never affects cuts
        self._stream = _Stream(ctx)
        self._blk = None                  # block taking the next read (no pipe)
        self._pos = 0
        # [block, start, n, retire, piped]: read, not yet yielded (piped: the
        # block counts against the pipe's PIPE_BLOCKS)
        self._segs = collections.deque()
        self._base = 0                    # absolute offset of the next chunk
        self._cuts = collections.deque()
        self._eof = False
        self._finished = False
        self._threaded = False
        self._pipe = None
        _iter_started()

    def __iter__(self) -> Iterator[bytes]:
        return self

    def _fill(self) -> None:
        while not self._cuts and not self._eof:
            if self._pipe is not None:
                item = self._pipe.get()
                if isinstance(item, BaseException):
                    raise item
                blk, p, n, retire, cuts, eof = item
                self._eof = eof
                self._segs.append([blk, p, n, retire, True])
                self._cuts.extend(cuts.tolist())
                continue
            if self._blk is None:
                self._blk, self._pos = _block(), 0
            blk, p = self._blk, self._pos
            n = _read_into(self._reader, blk.mv[p:])
            self._pos = p + n
            retire = not n or READ_SIZE - self._pos < MIN_READ
            if retire:
                self._blk = None
            # a large file (a read filled a whole block): the rest runs as a
            # pipeline (reader, feeder and this thread), this read included
            if n == READ_SIZE and os.environ.get("RCDC_READ_AHEAD", "1") != "0":
                self._threaded = True
                self._pipe = _Pipe(self._reader, self._stream, (blk, p, n, retire),
                                   _pipe_blocks(self._ctx))
                self._blk = None
                continue
            self._eof = not n
            cuts = self._stream.feed(blk.mv[p:p + n], self._eof)
            self._segs.append([blk, p, n, retire, False])
            self._cuts.extend(cuts.tolist())

    def _retire(self, seg) -> None:
        _release(seg[0])
        if seg[4] and self._pipe is not None:
            self._pipe.room.release()

    def _take(self, k: int) -> bytes:
        """The next k bytes read, releasing spent blocks.  The chunk is a new
        bytes object filled by memmove, which runs without the GIL (ctypes
        releases it around foreign calls), so the copy does not hold off the
        reader thread; the object is written before anyone else sees it."""
        segs = self._segs
        chunk = _new_bytes(None, k)
        dst, rem = id(chunk) + _BYTES_DATA, k
        while rem:  # usually one segment; a chunk may span reads and blocks
            if not segs:
                raise AssertionError("rcdc stream cut beyond the bytes fed")
            s = segs[0]
            t = min(rem, s[2])
            ctypes.memmove(dst, s[0].addr + s[1], t)
            dst += t
            rem -= t
            s[1] += t
            s[2] -= t
            if not s[2]:
                segs.popleft()
                if s[3]:
                    self._retire(s)
        while segs and not segs[0][2]:  # the EOF read's empty segment
            s = segs.popleft()
            if s[3]:
                self._retire(s)
        return chunk

    def _finish(self) -> None:
        """End of iteration (EOF, an error, or the caller dropping the
        iterator): stop the pipe's threads (a read or feed they are in
        finishes first) before the blocks can go back to the pool, then
        close the device stream."""
        if self._finished:
            return
        self._finished = True
        if self._pipe is not None:
            self._pipe.close()
            self._pipe = None
        self._blk = None
        self._segs.clear()
        self._stream.close()
        _iter_done()

    def close(self) -> None:
        """Stop early (the caller breaks out of its loop)."""
        self._finish()

    def __del__(self):
        try:
            self._finish()
        except Exception:  # interpreter shutdown
            pass

    def __next__(self) -> bytes:
        if self._finished:
            raise StopIteration
        try:
            self._fill()
        except RusticError:
            self._finish()
            raise
        if not self._cuts:
            self._finish()
            raise StopIteration
        end = self._cuts.popleft()
        chunk = self._take(end - self._base)
        self._base = end
        self.size_hint = max(self.size_hint - len(chunk), 0)
        return chunk


class FixedSizeChunkIter:
    """fixed_size.rs:41-70 -- cuts every ``size`` bytes (no hashing: host only)."""

    def __init__(self, size: int, reader, size_hint: int = 0):
        self._size = size
        self._reader = reader
        self.size_hint = size_hint
        self._finished = False

    def __iter__(self):
        return self

    def __next__(self) -> bytes:
        if self._finished:
            raise StopIteration
        out = bytearray()
        while len(out) < self._size:
            try:
                b = _read(self._reader, self._size - len(out))
            except RusticError:
                self._finished = True
                raise
            if not b:
                break
            out += b
        if len(out) < self._size:
            self._finished = True
        if not out:
            raise StopIteration
        self.size_hint = max(self.size_hint - len(out), 0)
        return bytes(out)


class ChunkIter:
    """chunker.rs:16-59 -- dispatch on ``ConfigFile.chunker``."""

    @staticmethod
    def from_config(config: ConfigFile, reader, size_hint: int = 0,
                    device: Optional[int] = None):
        if isinstance(reader, (bytes, bytearray, memoryview)):
            reader = io.BytesIO(bytes(reader))
        if config.get_chunker() == Chunker.Rabin:
            poly = config.poly()
            check_rabin_params(config.chunk_size(), config.chunk_min_size(),
                               config.chunk_max_size())
            ctx = Context.get(poly, config.chunk_min_size(), config.chunk_size(),
                              config.chunk_max_size(), device)
            return RabinChunkIter(ctx, reader, size_hint)
        return FixedSizeChunkIter(config.chunk_size(), reader, size_hint)


def fixed_cuts(n: int, size: int) -> np.ndarray:
    """Cut offsets of the FixedSize chunker via the C ABI (rcdc_fixed_cuts)."""
    cap = n // max(size, 1) + 1
    cuts = np.zeros(max(cap, 1), dtype=np.uint64)
    k = _lib.lib().rcdc_fixed_cuts(n, size, cuts.ctypes.data, cap)
    return cuts[:k]
