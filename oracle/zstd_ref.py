"""zstd checker -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's
cpu_baseline leg).  Never imported by the product path.

The reference compresses blobs with the `zstd` crate 0.13.3 over zstd-sys
2.0.16+zstd.1.5.7 (/root/reference/Cargo.lock:6115-6140):
`encode_all(data, level)` in backend/decrypt.rs:489-503 and `decode_all` in
decrypt.rs:71-95.  Neither the crate nor a Rust toolchain is here, and no
fixture in the reference holds a compressed blob (its test repositories are
version 1).  The contract between rustic and its compressor is the zstd
frame format (RFC 8878): whatever frames the device writes must decode, with
a standard decoder, to the blob's bytes, and carry its content size.  The
bytes of a compressed frame are library-version specific (libzstd 1.4.8
here vs 1.5.7 in the reference), so they are "parity unpinned" by design;
decoding is pinned.

Decoders used as checkers (two independent builds):
  - the system libzstd (libzstd.so.1, 1.4.8) through ctypes: ZSTD_decompress,
    ZSTD_decompressStream (decode_all's streaming decoder, with its window
    limit), ZSTD_getFrameContentSize, and ZSTD_compress for the CPU baseline
    (the library rustic itself links, at another version);
  - pyarrow's bundled zstd codec (cross-check).
"""
from __future__ import annotations

import ctypes
import ctypes.util
from typing import Optional

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("zstd") or "libzstd.so.1"
        L = ctypes.CDLL(name)
        sz, vp = ctypes.c_size_t, ctypes.c_void_p
        L.ZSTD_versionNumber.restype = ctypes.c_uint
        L.ZSTD_compressBound.restype = sz
        L.ZSTD_compressBound.argtypes = [sz]
        L.ZSTD_compress.restype = sz
        L.ZSTD_compress.argtypes = [vp, sz, vp, sz, ctypes.c_int]
        L.ZSTD_decompress.restype = sz
        L.ZSTD_decompress.argtypes = [vp, sz, vp, sz]
        L.ZSTD_isError.restype = ctypes.c_uint
        L.ZSTD_isError.argtypes = [sz]
        L.ZSTD_getErrorName.restype = ctypes.c_char_p
        L.ZSTD_getErrorName.argtypes = [sz]
        L.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong
        L.ZSTD_getFrameContentSize.argtypes = [vp, sz]
        L.ZSTD_findFrameCompressedSize.restype = sz
        L.ZSTD_findFrameCompressedSize.argtypes = [vp, sz]
        L.ZSTD_createDStream.restype = vp
        L.ZSTD_freeDStream.argtypes = [vp]
        L.ZSTD_initDStream.restype = sz
        L.ZSTD_initDStream.argtypes = [vp]
        L.ZSTD_decompressStream.restype = sz
        L.ZSTD_decompressStream.argtypes = [vp, vp, vp]
        _lib = L
    return _lib


def version() -> str:
    v = lib().ZSTD_versionNumber()
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}"


class ZstdError(ValueError):
    pass


def _check(r: int) -> int:
    L = lib()
    if L.ZSTD_isError(r):
        raise ZstdError(L.ZSTD_getErrorName(r).decode())
    return r


def content_size(frame: bytes) -> Optional[int]:
    """The frame header's content size (None if absent)."""
    v = lib().ZSTD_getFrameContentSize(frame, len(frame))
    if v >= (1 << 64) - 2:  # ZSTD_CONTENTSIZE_UNKNOWN / _ERROR
        if v == (1 << 64) - 2:
            raise ZstdError("not a zstd frame")
        return None
    return int(v)


def frame_size(frame: bytes) -> int:
    """Bytes of the first frame in `frame` (the decoder's own parse)."""
    return _check(lib().ZSTD_findFrameCompressedSize(frame, len(frame)))


def decompress(frame: bytes, size: Optional[int] = None) -> bytes:
    """decode_all of one frame with libzstd (rustic's decrypt.rs:71-95)."""
    if size is None:
        size = content_size(frame)
        if size is None:
            raise ZstdError("frame without content size")
    buf = ctypes.create_string_buffer(max(size, 1))
    n = _check(lib().ZSTD_decompress(buf, size, frame, len(frame)))
    return buf.raw[:n]


class _ZBuf(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


def decompress_stream(frame: bytes, step: int = 8192) -> bytes:
    """decode_all as rustic runs it: the zstd crate's streaming Decoder
    (ZSTD_decompressStream with libzstd's defaults, so frames asking for a
    window above 2^27 + 1 bytes are refused -- single-segment frames ask for
    their content size), read through `step`-byte output buffers (io::copy's
    8 KiB).  A frame whose content fits the first buffer takes libzstd's
    one-pass shortcut instead, which checks no window and refuses empty
    compressed blocks; larger ones go through the stage machine.  One frame;
    raises ZstdError."""
    L = lib()
    ds = L.ZSTD_createDStream()
    try:
        _check(L.ZSTD_initDStream(ds))
        src = ctypes.create_string_buffer(frame, len(frame))
        ib = _ZBuf(ctypes.cast(src, ctypes.c_void_p), len(frame), 0)
        dst = ctypes.create_string_buffer(step)
        out = []
        while True:
            ob = _ZBuf(ctypes.cast(dst, ctypes.c_void_p), step, 0)
            r = _check(L.ZSTD_decompressStream(ds, ctypes.byref(ob), ctypes.byref(ib)))
            out.append(dst.raw[:ob.pos])
            if r == 0:
                return b"".join(out)
            if ob.pos == 0 and ib.pos == len(frame):
                raise ZstdError("truncated frame")
    finally:
        L.ZSTD_freeDStream(ds)


def decompress_pyarrow(frame: bytes, size: int) -> bytes:
    import pyarrow as pa
    return pa.decompress(frame, decompressed_size=size, codec="zstd", asbytes=True)


def compress(data: bytes, level: int = 3) -> bytes:
    """libzstd's one-shot compression (the CPU baseline; encode_all's library)."""
    L = lib()
    cap = L.ZSTD_compressBound(len(data))
    buf = ctypes.create_string_buffer(cap)
    n = _check(L.ZSTD_compress(buf, cap, data, len(data), level))
    return buf.raw[:n]


def compress_into(dst_ptr: int, cap: int, src_ptr: int, n: int, level: int = 3) -> int:
    """ZSTD_compress between raw pointers (numpy buffers; for timing)."""
    return _check(lib().ZSTD_compress(dst_ptr, cap, src_ptr, n, level))


# ---- frame walking (block types and sizes; RFC 8878 3.1.1) -----------------

def blocks(frame: bytes):
    """[(type, block_size, last)] of a single-segment frame: 0 raw, 1 RLE,
    2 compressed.  Raises on anything else than this library's layout."""
    if frame[:4] != b"\x28\xb5\x2f\xfd":
        raise ZstdError("bad magic")
    fhd = frame[4]
    fcs_flag, single = fhd >> 6, (fhd >> 5) & 1
    if not single or fhd & 0x1F:
        raise ZstdError(f"unexpected frame header descriptor {fhd:#x}")
    pos = 5 + (1, 2, 4, 8)[fcs_flag]
    out = []
    while True:
        h = int.from_bytes(frame[pos:pos + 3], "little")
        last, tpe, size = h & 1, (h >> 1) & 3, h >> 3
        pos += 3
        out.append((tpe, size, bool(last)))
        pos += 1 if tpe == 1 else size
        if last:
            break
    if pos != len(frame):
        raise ZstdError(f"frame is {len(frame)} bytes, blocks end at {pos}")
    return out
