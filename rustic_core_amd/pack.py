"""Pack files on the device: the packer's byte work for blobs in HBM
(rcdc_pack_build in include/rcdc.h).

Reference: ``blob/packer.rs`` -- ``PackSizer`` (:65-200) decides how many
blobs go into a pack, ``BasicPacker::add_raw`` (:615-655) appends each sealed
blob and records its index entry, ``save`` / ``write_header`` (:505-510,
:693-735) append the sealed header and its u32 length; the header entries
are ``HeaderEntry`` (``repofile/packfile.rs:88-124``).  Here the grouping
runs on the host (``PackSizer``, ``group_blobs``) and one device call seals
every blob and header of a batch of packs into their final layout.  The pack
id (SHA-256 of the pack file, packer.rs:833) is the caller's.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .errors import status_error

MB = 1 << 20
MAX_SIZE = 4076 * MB   # packer.rs:58
MAX_COUNT = 10_000     # packer.rs:60

# rcdc_pack_blob / rcdc_pack (include/rcdc.h)
PACK_BLOB = np.dtype([("in_off", "<u8"), ("len", "<u4"), ("uncompressed_len", "<u4"),
                      ("type", "<u4"), ("pad", "<u4"), ("id", "u1", (32,)),
                      ("nonce", "u1", (16,))])
PACK = np.dtype([("out_off", "<u8"), ("blob0", "<u4"), ("nblobs", "<u4"),
                 ("header_nonce", "u1", (16,)), ("size", "<u8"), ("header_len", "<u4"),
                 ("pad", "<u4")])
assert PACK_BLOB.itemsize == 72 and PACK.itemsize == 48


class PackSizer:
    """packer.rs:65-200."""

    def __init__(self, default_size: int, grow_factor: int, size_limit: int, current_size: int,
                 min_percent: int, max_percent: int):
        self.default_size = default_size
        self.grow_factor = grow_factor
        self.size_limit = size_limit
        self.current_size = current_size
        self.min_packsize_tolerate_percent = min_percent
        self.max_packsize_tolerate_percent = max_percent

    @classmethod
    def from_config(cls, config, blob_type: int, current_size: int) -> "PackSizer":  # :96-108
        size, grow, limit = config.packsize(blob_type)
        lo, hi = config.packsize_ok_percents()
        return cls(size, grow, limit, current_size, lo, hi)

    @classmethod
    def fixed(cls, size: int) -> "PackSizer":  # :120-129
        return cls(size, 0, size, 0, 100, 100)

    def pack_size(self) -> int:  # :134-146
        if self.grow_factor == 0:
            size = self.default_size
        else:
            size = (math.isqrt(self.current_size) * self.grow_factor + self.default_size)
            size &= 0xFFFFFFFF  # u32 arithmetic
        return min(size, self.size_limit, MAX_SIZE)

    def is_too_small(self, size: int) -> bool:  # :162-167
        return size * 100 < self.pack_size() * self.min_packsize_tolerate_percent

    def is_too_large(self, size: int) -> bool:  # :175-180
        return size * 100 > self.pack_size() * self.max_packsize_tolerate_percent

    def size_ok(self, size: int) -> bool:  # :152-154
        return not self.is_too_small(size) and not self.is_too_large(size)

    def add_size(self, added: int) -> None:  # :191-193
        self.current_size += added


def header_entry_len(uncompressed_len: int) -> int:
    """HeaderEntry::length (packfile.rs:158-163): 37, or 41 compressed."""
    return 41 if uncompressed_len else 37


def group_blobs(lens: Sequence[int], sizer: PackSizer,
                uncompressed: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """Packs as (blob0, nblobs), in blob order, the way the packer fills them:
    add_raw appends a blob (len + 32 sealed bytes), then should_save
    (packer.rs:659-671) closes the pack at MAX_COUNT blobs or once its size
    reaches pack_size(); take_data (:749-758) adds the closed pack's
    PackHeaderRef::pack_size to the sizer.  (MAX_AGE, a wall-clock rule, is
    not modelled.)  The last pack holds the rest (finalize)."""
    return group_blobs_open(lens, sizer, uncompressed, finalize=True)[0]


def group_blobs_open(lens: Sequence[int], sizer: PackSizer,
                     uncompressed: Optional[Sequence[int]] = None,
                     finalize: bool = False) -> Tuple[List[Tuple[int, int]], int]:
    """group_blobs for a packer that stays open between calls (one Packer
    for the whole backup, packer.rs:659-671 / 749-750): returns the packs
    should_save closed and the index of the first blob of the still open
    pack (len(lens) if none).  The open pack's size is NOT added to the sizer
    (take_data has not run for it); with ``finalize`` it is closed too
    (Packer::finalize)."""
    # a pack at a time (pack_size() only changes when a pack closes): its
    # last blob is the first whose running sealed size reaches pack_size(),
    # or the MAX_COUNT-th (numpy over prefix sums, not a Python loop per blob)
    n_all = len(lens)
    sealed = np.asarray(lens, np.int64) + 32
    hdr_b = np.full(n_all, 37, np.int64)
    if uncompressed is not None:
        hdr_b = np.where(np.asarray(uncompressed, np.int64) > 0, 41, 37)
    cum = np.concatenate([np.zeros(1, np.int64), np.cumsum(sealed)])
    cumh = np.concatenate([np.zeros(1, np.int64), np.cumsum(hdr_b)])
    packs, b0 = [], 0
    while b0 < n_all:
        limit = cum[b0] + sizer.pack_size()
        i = int(np.searchsorted(cum, limit, side="left"))  # cum[i] >= limit: blobs b0..i-1
        e = min(max(i, b0 + 1), b0 + MAX_COUNT, n_all)       # one past the pack's last blob
        closed = cum[e] - cum[b0] >= sizer.pack_size() or e - b0 >= MAX_COUNT
        if not closed and not finalize:
            break  # should_save is false after the last blob: the pack stays open
        packs.append((b0, e - b0))
        sizer.add_size(int(cum[e] - cum[b0] + cumh[e] - cumh[b0]) + 32 + 4)
        b0 = e
    return packs, b0


def make_blobs(in_offs, lens, ids, nonces, types=None, uncompressed=None) -> np.ndarray:
    n = len(lens)
    b = np.zeros(n, PACK_BLOB)
    b["in_off"] = np.asarray(in_offs, np.uint64)
    b["len"] = np.asarray(lens, np.uint32)
    b["id"] = np.asarray(ids, np.uint8).reshape(n, 32)
    b["nonce"] = np.asarray(nonces, np.uint8).reshape(n, 16)
    if types is not None:
        b["type"] = np.asarray(types, np.uint32)
    if uncompressed is not None:
        b["uncompressed_len"] = np.asarray(uncompressed, np.uint32)
    return b


def pack_layout(blobs: np.ndarray, groups: Sequence[Tuple[int, int]], header_nonces,
                align: int = 1, raw: bool = False) -> Tuple[np.ndarray, int]:
    """rcdc_pack array for `groups`, packed back to back in one output
    buffer (each pack `align`-aligned); returns (packs, total bytes).
    ``raw``: blobs["len"] are sealed lengths already (build_packs raw)."""
    packs = np.zeros(len(groups), PACK)
    per = blobs["len"].astype(np.int64) + (0 if raw else 32) + \
        np.where(blobs["uncompressed_len"] > 0, 41, 37)
    cum = np.concatenate([np.zeros(1, np.int64), np.cumsum(per)])
    o = 0
    for k, (b0, n) in enumerate(groups):
        size = int(cum[b0 + n] - cum[b0]) + 32 + 4
        packs[k]["out_off"] = o
        packs[k]["blob0"] = b0
        packs[k]["nblobs"] = n
        o = (o + size + align - 1) // align * align
    packs["header_nonce"] = np.asarray(header_nonces, np.uint8).reshape(len(groups), 16)
    return packs, o


def build_packs(ctx, key: bytes, d_in: int, blobs: np.ndarray, packs: np.ndarray, d_out: int,
                out_len: int, hip_stream: Optional[int] = None, raw: bool = False) -> np.ndarray:
    """rcdc_pack_build: fills packs["size"], packs["header_len"] and returns
    each blob's offset in its pack (IndexBlob location.offset; length =
    len + 32).  ``raw`` (rcdc_pack_build_raw, packer.rs add_raw): the blobs
    at in_off are sealed already and blobs["len"] is their sealed length;
    they are copied, only the headers are sealed."""
    blobs = np.ascontiguousarray(blobs, PACK_BLOB)
    if not (packs.flags["C_CONTIGUOUS"] and packs.dtype == PACK):
        raise TypeError("packs must be a C-contiguous PACK array (it receives the sizes)")
    offs = np.zeros(max(len(blobs), 1), np.uint32)
    kb = (ctypes.c_uint8 * 64).from_buffer_copy(bytes(key))
    fn = _lib.lib().rcdc_pack_build_raw if raw else _lib.lib().rcdc_pack_build
    st = fn(ctx.handle, kb, ctypes.c_void_p(d_in), blobs.ctypes.data, len(blobs),
            packs.ctypes.data, len(packs), ctypes.c_void_p(d_out), int(out_len),
            offs.ctypes.data, ctypes.c_void_p(hip_stream or 0))
    if st:
        raise status_error(st, _lib.last_error())
    return offs[:len(blobs)]


def build_packs_multi(ctx, key: bytes, d_ins: Sequence[int], blobs: np.ndarray,
                      packs: np.ndarray, d_out: int, out_len: int,
                      hip_stream: Optional[int] = None) -> np.ndarray:
    """rcdc_pack_build_raw_multi: build_packs(raw=True) over sealed blobs in
    several device buffers, blobs["pad"] selecting d_ins[pad]."""
    blobs = np.ascontiguousarray(blobs, PACK_BLOB)
    if not (packs.flags["C_CONTIGUOUS"] and packs.dtype == PACK):
        raise TypeError("packs must be a C-contiguous PACK array (it receives the sizes)")
    offs = np.zeros(max(len(blobs), 1), np.uint32)
    kb = (ctypes.c_uint8 * 64).from_buffer_copy(bytes(key))
    srcs = (ctypes.c_void_p * max(len(d_ins), 1))(*[int(p) for p in d_ins])
    st = _lib.lib().rcdc_pack_build_raw_multi(
        ctx.handle, kb, ctypes.cast(srcs, ctypes.c_void_p), len(d_ins), blobs.ctypes.data,
        len(blobs), packs.ctypes.data, len(packs), ctypes.c_void_p(d_out), int(out_len),
        offs.ctypes.data, ctypes.c_void_p(hip_stream or 0))
    if st:
        raise status_error(st, _lib.last_error())
    return offs[:len(blobs)]


COPY_REF = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("len", "<u8"), ("src", "<u4"),
                     ("pad", "<u4")])
assert COPY_REF.itemsize == 32


def copy_ranges(ctx, d_ins: Sequence[int], src, in_offs, lens, out_offs, d_out: int,
                hip_stream: Optional[int] = None) -> None:
    """rcdc_copy_ranges: bytes [in_off, +len) of d_ins[src] to out_off of d_out."""
    n = len(lens)
    refs = np.zeros(n, COPY_REF)
    refs["in_off"], refs["out_off"], refs["len"] = in_offs, out_offs, lens
    refs["src"] = src
    srcs = (ctypes.c_void_p * max(len(d_ins), 1))(*[int(p) for p in d_ins])
    st = _lib.lib().rcdc_copy_ranges(ctx.handle, ctypes.cast(srcs, ctypes.c_void_p), len(d_ins),
                                     refs.ctypes.data, n, ctypes.c_void_p(d_out),
                                     ctypes.c_void_p(hip_stream or 0))
    if st:
        raise status_error(st, _lib.last_error())


def index_entries(blobs: np.ndarray, packs: np.ndarray, offsets: np.ndarray):
    """IndexPack blobs per pack (indexfile.rs IndexBlob): [(id, type, offset,
    length, uncompressed_length or None)]."""
    out = []
    for p in packs:
        b0, n = int(p["blob0"]), int(p["nblobs"])
        out.append([(bytes(blobs[i]["id"]), int(blobs[i]["type"]), int(offsets[i]),
                     int(blobs[i]["len"]) + 32,
                     int(blobs[i]["uncompressed_len"]) or None) for i in range(b0, b0 + n)])
    return out


def random_nonces(n: int) -> np.ndarray:
    """One fresh nonce per blob (aespoly1305.rs:120-121 draws from the OS RNG)."""
    return np.frombuffer(os.urandom(16 * n), np.uint8).reshape(n, 16)
