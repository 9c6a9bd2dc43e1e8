"""Blob compression on the device: the zstd step of rustic_core's
``DecryptBackend::encrypt_data`` (crates/core/src/backend/decrypt.rs:478-506:
``encode_all(data, level)`` before ``Key::encrypt_data`` when the repository
is version 2, configfile.rs:177-186) over blobs already in HBM
(rcdc_zstd_compress in include/rcdc.h).

Each blob becomes one zstd frame (RFC 8878) that any zstd decoder reads back
-- rustic's own ``decode_all`` (decrypt.rs:71-95) included.  ``compress_blobs``
is the batch form (the packer compresses every new blob,
blob/packer.rs:268-270); ``encode_all`` keeps the byte-in/byte-out signature
for one blob; ``process_blobs`` is ``process_data`` (decrypt.rs:566-572) for a
batch: compress, then seal, with the returned ``(data_len,
uncompressed_length)`` the index needs.  No CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from .chunker import Context
from .errors import ErrorKind, RusticError, status_error

# rcdc_zstd_ref (include/rcdc.h)
ZSTD_REF = np.dtype([("in_off", "<u8"), ("len", "<u8"), ("out_off", "<u8")])
assert ZSTD_REF.itemsize == 24

# zstd's level range (decrypt.rs:20-24, zstd::compression_level_range)
MIN_LEVEL, MAX_LEVEL = -(1 << 17), 22


def zstd_bound(n: int) -> int:
    """Worst-case frame bytes of an n-byte blob."""
    return int(_lib.lib().rcdc_zstd_bound(int(n)))


def frame_layout(lens, align: int = 16):
    """out_offs for frames of blobs of ``lens`` at their worst-case size."""
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o = (o + zstd_bound(int(n)) + align - 1) // align * align
    return np.array(offs, np.uint64), o


def make_refs(in_offs, lens, out_offs) -> np.ndarray:
    refs = np.zeros(len(lens), ZSTD_REF)
    refs["in_off"] = np.asarray(in_offs, np.uint64)
    refs["len"] = np.asarray(lens, np.uint64)
    refs["out_off"] = np.asarray(out_offs, np.uint64)
    return refs


def compress_blobs(ctx: Context, d_in: int, refs: np.ndarray, d_out: int, level: int = 0,
                   hip_stream: Optional[int] = None) -> np.ndarray:
    """Frames of every blob of ``refs`` into d_out; returns their lengths."""
    refs = np.ascontiguousarray(refs, ZSTD_REF)
    out_lens = np.zeros(max(len(refs), 1), np.uint64)
    st = _lib.lib().rcdc_zstd_compress(ctx.handle, int(level), ctypes.c_void_p(d_in),
                                       refs.ctypes.data, len(refs), ctypes.c_void_p(d_out),
                                       out_lens.ctypes.data, ctypes.c_void_p(hip_stream or 0))
    if st:
        raise status_error(st, _lib.last_error())
    return out_lens[:len(refs)]


def _ctx(device: int) -> Context:
    from .crypto import _ctx as c
    return c(device)


def encode_all(data: bytes, level: int = 0, device: int = 0) -> bytes:
    """zstd::encode_all for one blob, through HBM (decrypt.rs:493)."""
    import torch
    n = len(data)
    dev = torch.device("cuda", device)
    src = torch.zeros(n + 4, dtype=torch.uint8)
    if n:
        src[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    d_in = src.to(dev)
    d_out = torch.empty(zstd_bound(n), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        s = torch.cuda.current_stream(dev).cuda_stream
        ln = compress_blobs(_ctx(device), d_in.data_ptr(), make_refs([0], [n], [0]),
                            d_out.data_ptr(), level, s)
    return d_out[:int(ln[0])].cpu().numpy().tobytes()


def process_blobs(key, d_in: int, in_offs, lens, level: Optional[int] = 0, nonces=None,
                  device: int = 0):
    """DecryptWriteBackend::process_data (decrypt.rs:566-572) for a batch of
    blobs in HBM: compress (level not None) and seal.  Returns (sealed
    device tensor, sealed offsets, sealed lengths, data_len,
    uncompressed_length) -- uncompressed_length is 0 where nothing was
    compressed (``None`` in the reference)."""
    import torch
    from .crypto import make_refs as aead_refs, sealed_layout
    from .pack import random_nonces
    lens = np.asarray(lens, np.uint64)
    if len(lens) and int(lens.max()) > 0xFFFFFFFF:  # decrypt.rs:479-487
        raise RusticError(ErrorKind.Internal, "Failed to convert data length to u32.")
    n = len(lens)
    dev = torch.device("cuda", device)
    ctx = _ctx(device)
    nonces = random_nonces(n) if nonces is None else nonces
    with torch.cuda.device(dev):
        s = torch.cuda.current_stream(dev).cuda_stream
        if level is None:
            src, src_offs, src_lens = d_in, np.asarray(in_offs, np.uint64), lens
            keep = None
        else:
            f_offs, total = frame_layout(lens)
            keep = torch.empty(max(total, 1) + 16, dtype=torch.uint8, device=dev)
            src_lens = compress_blobs(ctx, d_in, make_refs(in_offs, lens, f_offs),
                                      keep.data_ptr(), level, s)
            src, src_offs = keep.data_ptr(), f_offs
        s_offs, s_total = sealed_layout(src_lens)
        out = torch.empty(max(s_total, 1), dtype=torch.uint8, device=dev)
        key.seal_blobs(src, aead_refs(src_offs, src_lens, s_offs, nonces), out.data_ptr(), s, ctx)
        torch.cuda.synchronize(dev)
    del keep
    ulen = lens.copy() if level is not None else np.zeros(n, np.uint64)
    return out, s_offs, np.asarray(src_lens, np.uint64) + 32, lens, ulen
