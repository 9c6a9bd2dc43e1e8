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

# rcdc_zstd_check_ref (include/rcdc.h)
ZSTD_CHECK_REF = np.dtype([("frame_off", "<u8"), ("frame_len", "<u8"), ("data_off", "<u8"),
                           ("data_len", "<u8")])
assert ZSTD_CHECK_REF.itemsize == 32

# frame check status (rcdc_zstd_check)
CHECK_OK, CHECK_MISMATCH, CHECK_CORRUPT = 0, 1, 2

# zstd's level range (decrypt.rs:20-24, zstd::compression_level_range)
MIN_LEVEL, MAX_LEVEL = -(1 << 17), 22


def zstd_bound(n: int) -> int:
    """Worst-case frame bytes of an n-byte blob."""
    return int(_lib.lib().rcdc_zstd_bound(int(n)))


def zstd_bounds(lens) -> np.ndarray:
    """rcdc_zstd_bound of every length (numpy; the same formula)."""
    lens = np.asarray(lens, np.int64)
    nblk = np.maximum((lens + (128 << 10) - 1) // (128 << 10), 1)
    return lens + 3 * nblk + np.where(lens > (1 << 27), 10, 9)  # + the window byte


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


def check_frames(ctx: Context, d_frames: int, frame_offs, frame_lens, d_data: int, data_offs,
                 data_lens, hip_stream: Optional[int] = None, stored: bool = False) -> np.ndarray:
    """Decode every frame on the device and compare it with its blob
    (rcdc_zstd_check): per frame 0 = equal, 1 = other bytes or length,
    2 = malformed / not readable here.  ``stored``: the "frames" are plain
    bytes (uncompressed blobs), compared as they are."""
    n = len(frame_lens)
    refs = np.zeros(max(n, 1), ZSTD_CHECK_REF)
    refs["frame_off"][:n] = np.asarray(frame_offs, np.uint64)
    refs["frame_len"][:n] = np.asarray(frame_lens, np.uint64)
    refs["data_off"][:n] = np.asarray(data_offs, np.uint64)
    refs["data_len"][:n] = np.asarray(data_lens, np.uint64)
    status = np.zeros(max(n, 1), np.uint32)
    st = _lib.lib().rcdc_zstd_check(ctx.handle, ctypes.c_void_p(d_frames), ctypes.c_void_p(d_data),
                                    refs.ctypes.data, n, 1 if stored else 0, status.ctypes.data,
                                    ctypes.c_void_p(hip_stream or 0))
    if st:
        raise status_error(st, _lib.last_error())
    return status[:n]


VERIFY_MESSAGE = ("Verification failed: After decrypting and decompressing the data changed! "
                  "The data may be corrupted.")  # decrypt.rs:519-521


def verify_sealed(ctx: Context, key, d_sealed: int, sealed_offs, sealed_lens, d_data: int,
                  data_offs, data_lens, compressed: bool, hip_stream: Optional[int] = None,
                  scratch=None) -> None:
    """very_data (decrypt.rs:508-529) for a batch: open every sealed blob on
    the device (MAC checked), then decode its frame (or take the plaintext
    when not compressed) and compare it with the input bytes.  Raises
    ErrorKind.Verification on the first blob that does not come back."""
    import torch
    from .crypto import make_refs as aead_refs, sealed_layout
    n = len(sealed_lens)
    if n == 0:
        return
    plain_lens = np.asarray(sealed_lens, np.uint64) - 32
    p_offs, total = sealed_layout(plain_lens)  # 16-aligned plaintexts
    dev = torch.device("cuda", ctx.device)
    if scratch is None or scratch.numel() < total + 64:
        scratch = torch.empty(int(total) + 64, dtype=torch.uint8, device=dev)
    st = key.open_blobs(d_sealed, aead_refs(sealed_offs, sealed_lens, p_offs), scratch.data_ptr(),
                        hip_stream, ctx)
    bad = np.nonzero(st)[0]
    if len(bad):
        raise RusticError(ErrorKind.Verification,
                          f"{VERIFY_MESSAGE} (blob {int(bad[0])}: MAC check failed)")
    # compressed: decode each frame; else the plaintext is compared as is
    cs = check_frames(ctx, scratch.data_ptr(), p_offs, plain_lens, d_data, data_offs, data_lens,
                      hip_stream, stored=not compressed)
    bad = np.nonzero(cs)[0]
    if len(bad):
        raise RusticError(ErrorKind.Verification,
                          f"{VERIFY_MESSAGE} (blob {int(bad[0])}: status {int(cs[bad[0]])})")


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
                  device: int = 0, extra_verify: bool = True):
    """DecryptWriteBackend::process_data (decrypt.rs:566-572) for a batch of
    blobs in HBM: compress (level not None), seal, and -- with
    ``extra_verify`` (the reference's default, configfile.rs:198) -- open and
    decode every sealed blob again and compare it with the input
    (``very_data``, decrypt.rs:508-529; ErrorKind.Verification).  Returns
    (sealed device tensor, sealed offsets, sealed lengths, data_len,
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
        if extra_verify:
            verify_sealed(ctx, key, out.data_ptr(), s_offs, np.asarray(src_lens, np.uint64) + 32,
                          d_in, in_offs, lens, level is not None, s)
        torch.cuda.synchronize(dev)
    del keep
    ulen = lens.copy() if level is not None else np.zeros(n, np.uint64)
    return out, s_offs, np.asarray(src_lens, np.uint64) + 32, lens, ulen
