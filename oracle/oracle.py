"""ctypes front-end of the CPU ORACLE (``oracle/libcdc_ref.so``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` -- as the checker, never as the
thing measured or shipped.  The product (``rustic_core_amd``) never imports
this module.

The C code restates ``crates/core/src/chunker/rabin.rs:107-191`` and the
rustic_cdc 0.3.1 Rabin64 arithmetic (see ``oracle/cdc_ref.h`` for the
file:line map and the parity pin).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libcdc_ref.so")

DEFAULT_POLY = 0x003DA3358B4DC173  # rabin.rs:336 test polynomial
KiB = 1024
MiB = 1024 * KiB
DEFAULT_MIN = 512 * KiB  # configfile.rs:39
DEFAULT_AVG = 1 * MiB    # configfile.rs:37
DEFAULT_MAX = 8 * MiB    # configfile.rs:41


def build() -> str:
    """Compile the oracle with its Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


class _Tables(ctypes.Structure):
    _fields_ = [
        ("out_table", ctypes.c_uint64 * 256),
        ("mod_table", ctypes.c_uint64 * 256),
        ("degree", ctypes.c_int),
        ("shift", ctypes.c_int),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in ("cdc_ref.c", "crypto_ref.c")]
        if not os.path.exists(_SO) or any(
            os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(_SO) for src in srcs
        ):
            build()
        L = ctypes.CDLL(_SO)
        u64, sz, p = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
        L.cdc_ref_tables_init.argtypes = [ctypes.POINTER(_Tables), u64]
        L.cdc_ref_tables_init.restype = ctypes.c_int
        L.cdc_ref_check_params.argtypes = [u64, u64, u64]
        L.cdc_ref_check_params.restype = ctypes.c_int
        L.cdc_ref_chunk.argtypes = [ctypes.POINTER(_Tables), p, sz, u64, u64, u64,
                                    ctypes.c_int, p, sz]
        L.cdc_ref_chunk.restype = sz
        L.cdc_ref_chunk_owned.argtypes = [ctypes.POINTER(_Tables), p, sz, u64, u64,
                                          u64, p, sz]
        L.cdc_ref_chunk_owned.restype = sz
        L.cdc_ref_chunk_owned_reads.argtypes = [ctypes.POINTER(_Tables), p, sz, u64, u64,
                                                u64, u64, p, sz]
        L.cdc_ref_chunk_owned_reads.restype = sz
        L.cdc_ref_chunk_many_owned.argtypes = [ctypes.POINTER(_Tables), p, p, p, sz,
                                               u64, u64, u64, ctypes.c_int, p]
        L.cdc_ref_chunk_many_owned.restype = u64
        L.cdc_ref_chunk_many_cuts.argtypes = [ctypes.POINTER(_Tables), p, p, p, sz, u64, u64,
                                              u64, ctypes.c_int, p, p, p, p]
        L.cdc_ref_chunk_many_cuts.restype = u64
        L.cdc_ref_fixed.argtypes = [sz, u64, p, sz]
        L.cdc_ref_fixed.restype = sz
        L.cdc_ref_candidates.argtypes = [ctypes.POINTER(_Tables), p, sz, u64, sz, sz, p]
        L.cdc_ref_candidates.restype = None
        L.cdc_ref_stdrng_fill.argtypes = [u64, p, sz]
        L.cdc_ref_stdrng_fill.restype = None
        L.cdc_ref_stdrng_fill_at.argtypes = [u64, u64, p, sz]
        L.cdc_ref_stdrng_fill_at.restype = None
        L.crypto_ref_seal.argtypes = [p, p, p, sz, p]
        L.crypto_ref_seal.restype = None
        L.crypto_ref_open.argtypes = [p, p, sz, p]
        L.crypto_ref_open.restype = ctypes.c_int
        L.crypto_ref_aes_expand.argtypes = [p, ctypes.c_int, p]
        L.crypto_ref_aes_expand.restype = ctypes.c_int
        L.crypto_ref_aes_encrypt.argtypes = [p, ctypes.c_int, p, p]
        L.crypto_ref_aes_encrypt.restype = None
        L.crypto_ref_poly1305.argtypes = [p, p, p, sz, p]
        L.crypto_ref_poly1305.restype = None
        _lib = L
    return _lib


_tables_cache: dict = {}


def tables(poly: int = DEFAULT_POLY) -> _Tables:
    t = _tables_cache.get(poly)
    if t is None:
        t = _Tables()
        if lib().cdc_ref_tables_init(ctypes.byref(t), poly) != 0:
            raise ValueError(f"unsupported polynomial {poly:#x}")
        _tables_cache[poly] = t
    return t


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def chunk_cuts(data, poly=DEFAULT_POLY, min_size=DEFAULT_MIN, avg=DEFAULT_AVG,
               max_size=DEFAULT_MAX, prefill64: bool = False) -> np.ndarray:
    """End offsets of every chunk (ChunkIter::next semantics, rabin.rs:107-191)."""
    a = _as_u8(data)
    n = a.size
    cap = n // max(min_size, 1) + 2
    cuts = np.zeros(cap, dtype=np.uint64)
    k = lib().cdc_ref_chunk(ctypes.byref(tables(poly)), _ptr(a), n, min_size, avg,
                            max_size, int(prefill64), _ptr(cuts), cap)
    assert k <= cap
    return cuts[:k].copy()


class ReferenceUnderflow(ArithmeticError):
    """rabin.rs:124 `min_size -= open_buf_len` would underflow (min below the
    up-to-4095 read-ahead bytes of the 4 KiB buffer, rabin.rs:12): the
    reference panics under debug assertions and wraps in release."""


UNDERFLOW = (1 << 64) - 1  # CDC_REF_UNDERFLOW


def chunk_cuts_owned(data, poly=DEFAULT_POLY, min_size=DEFAULT_MIN, avg=DEFAULT_AVG,
                     max_size=DEFAULT_MAX, read_seed: int = 0) -> np.ndarray:
    """Same cuts, reference-equivalent work (owned chunk buffers, 4 KiB reads,
    rabin.rs:110-191).  read_seed != 0: every reader read() returns a
    pseudo-random 1..n bytes (a pipe-like reader) instead of filling the
    request.  Raises ReferenceUnderflow where the reference would underflow."""
    a = _as_u8(data)
    n = a.size
    cap = n // max(min_size, 1) + 2
    cuts = np.zeros(cap, dtype=np.uint64)
    k = lib().cdc_ref_chunk_owned_reads(ctypes.byref(tables(poly)), _ptr(a), n, min_size,
                                        avg, max_size, read_seed, _ptr(cuts), cap)
    if k == UNDERFLOW:
        raise ReferenceUnderflow(f"rabin.rs:124 underflow at min={min_size}")
    return cuts[:k].copy()


def chunk_many_owned(arena: np.ndarray, offs, lens, poly=DEFAULT_POLY,
                     min_size=DEFAULT_MIN, avg=DEFAULT_AVG, max_size=DEFAULT_MAX,
                     nthreads: int = 1) -> np.ndarray:
    """Chunk many files in parallel (per-file threads, archiver.rs:195). Returns counts."""
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    counts = np.zeros(offs.size, dtype=np.uint64)
    lib().cdc_ref_chunk_many_owned(ctypes.byref(tables(poly)), _ptr(arena), _ptr(offs),
                                   _ptr(lens), offs.size, min_size, avg, max_size,
                                   nthreads, _ptr(counts))
    return counts


def chunk_many_cuts(arena: np.ndarray, offs, lens, poly=DEFAULT_POLY,
                    min_size=DEFAULT_MIN, avg=DEFAULT_AVG, max_size=DEFAULT_MAX,
                    nthreads: int = 1) -> list:
    """Cut lists of many files (reference-equivalent work, per-file threads as
    archiver.rs:195): file i = arena[offs[i], offs[i] + lens[i]).  The parity
    checker of whole device batches."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8).reshape(-1)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    for o, n in zip(offs, lens):
        assert int(o) + int(n) <= arena.size
    caps = lens // np.uint64(max(min_size, 1)) + np.uint64(2)
    base = np.concatenate([np.zeros(1, np.uint64), np.cumsum(caps)[:-1]]).astype(np.uint64)
    cuts = np.zeros(int(caps.sum()) if caps.size else 1, dtype=np.uint64)
    counts = np.zeros(offs.size, dtype=np.uint64)
    lib().cdc_ref_chunk_many_cuts(ctypes.byref(tables(poly)), _ptr(arena), _ptr(offs),
                                  _ptr(lens), offs.size, min_size, avg, max_size, nthreads,
                                  _ptr(counts), _ptr(cuts), _ptr(base), _ptr(caps))
    out = []
    for i in range(offs.size):
        k = int(counts[i])
        assert k <= int(caps[i])
        out.append(cuts[int(base[i]):int(base[i]) + k].copy())
    return out


def fixed_cuts(n: int, size: int) -> np.ndarray:
    cap = n // size + 2
    cuts = np.zeros(cap, dtype=np.uint64)
    k = lib().cdc_ref_fixed(n, size, _ptr(cuts), cap)
    return cuts[:k].copy()


def candidates(data, first: int, count: int, poly=DEFAULT_POLY,
               mask: int = DEFAULT_AVG - 1) -> np.ndarray:
    """flags[i] = fp(data[p-64:p]) & mask == 0 for p = first + i."""
    a = _as_u8(data)
    assert first >= 64 and first + count - 1 <= a.size
    flags = np.zeros(count, dtype=np.uint8)
    lib().cdc_ref_candidates(ctypes.byref(tables(poly)), _ptr(a), a.size, mask, first,
                             count, _ptr(flags))
    return flags


def check_params(avg: int, min_size: int, max_size: int) -> bool:
    return lib().cdc_ref_check_params(avg, min_size, max_size) == 0


def stdrng_bytes(seed: int, n: int, skip: int = 0) -> np.ndarray:
    """rand 0.10 ``StdRng::seed_from_u64(seed).fill_bytes`` (optionally from byte ``skip``)."""
    assert skip % 64 == 0
    buf = np.empty(n, dtype=np.uint8)
    lib().cdc_ref_stdrng_fill_at(seed, skip, _ptr(buf), n)
    return buf


def table_arrays(poly: int = DEFAULT_POLY):
    t = tables(poly)
    return (np.array(t.out_table[:], dtype=np.uint64),
            np.array(t.mod_table[:], dtype=np.uint64), t.degree, t.shift)


# ------------------------------------------------------------ blob encryption
# rustic Key::encrypt_data / decrypt_data (crates/core/src/crypto/aespoly1305.rs:88-135)
# restated in oracle/crypto_ref.c (aes256ctr_poly1305aes 0.2.1 = the restic format).
def _buf(b) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else \
        np.ascontiguousarray(b, dtype=np.uint8).reshape(-1)


def aes_encrypt_block(key: bytes, block: bytes) -> bytes:
    """One AES-128/256 block encryption (FIPS-197)."""
    rk = np.zeros(60, np.uint32)
    k = _buf(key)
    nr = lib().crypto_ref_aes_expand(_ptr(k), len(key) // 4, _ptr(rk))
    out = np.zeros(16, np.uint8)
    lib().crypto_ref_aes_encrypt(_ptr(rk), nr, _ptr(_buf(block)), _ptr(out))
    return out.tobytes()


def poly1305(r: bytes, s: bytes, msg: bytes) -> bytes:
    out = np.zeros(16, np.uint8)
    m = _buf(msg) if len(msg) else np.zeros(1, np.uint8)
    lib().crypto_ref_poly1305(_ptr(_buf(r)), _ptr(_buf(s)), _ptr(m), len(msg), _ptr(out))
    return out.tobytes()


def seal(key: bytes, nonce: bytes, data) -> bytes:
    """nonce || AES-256-CTR ciphertext || Poly1305-AES tag."""
    d = _buf(data) if len(data) else np.zeros(1, np.uint8)
    n = len(data)
    out = np.zeros(n + 32, np.uint8)
    lib().crypto_ref_seal(_ptr(_buf(key)), _ptr(_buf(nonce)), _ptr(d), n, _ptr(out))
    return out.tobytes()


class MacMismatch(ValueError):
    """decrypt_data: MAC check failed (ErrorKind::Cryptography, aespoly1305.rs:97-108)."""


def open_(key: bytes, data) -> bytes:
    d = _buf(data)
    out = np.zeros(max(d.size - 32, 1), np.uint8)
    st = lib().crypto_ref_open(_ptr(_buf(key)), _ptr(d), d.size, _ptr(out))
    if st == 2:
        raise ValueError("data too short")
    if st == 1:
        raise MacMismatch("MAC check failed")
    return out[:d.size - 32].tobytes()


# ---- pack files (test checker): blob/packer.rs:615-655 (add_raw),
# :693-735 (save / write_header), repofile/packfile.rs:88-124 (HeaderEntry),
# :355-372 (PackHeaderRef::size / pack_size) ---------------------------------

def pack_header_entry(tpe: int, sealed_len: int, blob_id: bytes,
                      uncompressed_len: int = 0) -> bytes:
    """HeaderEntry, little-endian: magic 0 Data / 1 Tree (+ u32 length + id),
    2 CompData / 3 CompTree (+ u32 length + u32 raw length + id)."""
    out = bytes([tpe + (2 if uncompressed_len else 0)]) + sealed_len.to_bytes(4, "little")
    if uncompressed_len:
        out += uncompressed_len.to_bytes(4, "little")
    return out + bytes(blob_id)


def pack_file(key: bytes, blobs, header_nonce: bytes):
    """blobs: (type, data, id, nonce, uncompressed_len) in pack order.
    Returns (pack bytes, [(offset, length)] per blob): the blobs sealed back
    to back, the sealed header, then its length as u32 LE."""
    body, index, off, header = [], [], 0, b""
    for tpe, data, bid, nonce, ulen in blobs:
        sealed = seal(key, nonce, data)
        body.append(sealed)
        index.append((off, len(sealed)))
        header += pack_header_entry(tpe, len(sealed), bid, ulen)
        off += len(sealed)
    sh = seal(key, header_nonce, header)
    return b"".join(body) + sh + len(sh).to_bytes(4, "little"), index


def parse_pack(key: bytes, pack: bytes):
    """PackHeader::from_binary over the decrypted header
    (packfile.rs:207-220): [(type, offset, length, uncompressed_len, id)]."""
    hlen = int.from_bytes(pack[-4:], "little")
    header = open_(key, pack[-4 - hlen:-4])
    out, pos, off = [], 0, 0
    while pos < len(header):
        t = header[pos]
        length = int.from_bytes(header[pos + 1:pos + 5], "little")
        if t in (0, 1):
            ulen, bid, pos = 0, header[pos + 5:pos + 37], pos + 37
        else:
            ulen = int.from_bytes(header[pos + 5:pos + 9], "little")
            bid, pos = header[pos + 9:pos + 41], pos + 41
        out.append((t & 1, off, length, ulen, bid))
        off += length
    return out
