"""Blob encryption on the device: rustic_core's ``Key`` (crates/core/src/crypto/
aespoly1305.rs:15-135) over blobs already in HBM (rcdc_aead_* in include/rcdc.h).

A sealed blob is ``nonce(16) || AES-256-CTR(data) || Poly1305-AES tag(16)``
(the restic format of aes256ctr_poly1305aes 0.2.1).  ``seal_blobs`` /
``open_blobs`` take a batch of blob references into a device arena -- the
packer's per-blob ``encrypt_data`` (blob/packer.rs:268-270) and the restore
path's ``decrypt_data`` (backend/decrypt.rs:566-572) -- and run on the GPU;
``encrypt_data`` / ``decrypt_data`` keep the reference's byte-in/byte-out
signature for one blob (the bytes go through HBM).  No CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from . import _lib
from .chunker import (Context, DEFAULT_CHUNK_MAX_SIZE, DEFAULT_CHUNK_MIN_SIZE,
                      DEFAULT_CHUNK_SIZE)
from .errors import ErrorKind, RusticError, status_error

# rcdc_aead_ref (include/rcdc.h)
AEAD_REF = np.dtype([("in_off", "<u8"), ("len", "<u8"), ("out_off", "<u8"),
                     ("nonce", "u1", (16,))])
assert AEAD_REF.itemsize == 40

# rustic's repository polynomial is irrelevant to encryption; any valid
# context serves as the device/stream holder
_POLY = 0x003DA3358B4DC173


def _ctx(device: int = 0) -> Context:
    return Context.get(_POLY, DEFAULT_CHUNK_MIN_SIZE, DEFAULT_CHUNK_SIZE,
                       DEFAULT_CHUNK_MAX_SIZE, device=device)


def make_refs(in_offs, lens, out_offs, nonces=None) -> np.ndarray:
    """Array of rcdc_aead_ref; ``nonces`` (n x 16 bytes) only for sealing."""
    n = len(lens)
    refs = np.zeros(n, AEAD_REF)
    refs["in_off"] = np.asarray(in_offs, np.uint64)
    refs["len"] = np.asarray(lens, np.uint64)
    refs["out_off"] = np.asarray(out_offs, np.uint64)
    if nonces is not None:
        refs["nonce"] = np.frombuffer(bytes(nonces), np.uint8).reshape(n, 16) \
            if isinstance(nonces, (bytes, bytearray)) else np.asarray(nonces, np.uint8)
    return refs


def sealed_layout(lens, align: int = 16):
    """out_offs of sealed blobs packed back to back (each 16-byte aligned)."""
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o = (o + int(n) + 32 + align - 1) // align * align
    return np.array(offs, np.uint64), o


class Key:
    """aespoly1305.rs:15-24: 32-byte AES-256 key || 16-byte k || 16-byte r."""

    def __init__(self, key: bytes):
        key = bytes(key)
        if len(key) != 64:
            raise RusticError(ErrorKind.InvalidInput, "key must be 64 bytes")
        self._key = key
        self._kbuf = (ctypes.c_uint8 * 64).from_buffer_copy(key)

    @classmethod
    def new(cls) -> "Key":  # :31-41 (random key)
        return cls(os.urandom(64))

    @classmethod
    def from_slice(cls, key: bytes) -> "Key":  # :43-53
        return cls(key)

    @classmethod
    def from_keys(cls, encrypt: bytes, k: bytes, r: bytes) -> "Key":  # :55-64
        return cls(bytes(encrypt) + bytes(k) + bytes(r))

    def to_keys(self):  # :66-75
        return self._key[:32], self._key[32:48], self._key[48:]

    # ---- batches in HBM -------------------------------------------------
    def seal_blobs(self, d_in: int, refs: np.ndarray, d_out: int,
                   hip_stream: Optional[int] = None, ctx: Optional[Context] = None) -> None:
        refs = np.ascontiguousarray(refs, AEAD_REF)
        c = ctx or _ctx()
        st = _lib.lib().rcdc_aead_seal(c.handle, self._kbuf, ctypes.c_void_p(d_in),
                                       refs.ctypes.data, len(refs), ctypes.c_void_p(d_out),
                                       ctypes.c_void_p(hip_stream or 0))
        if st:
            raise status_error(st, _lib.last_error())

    def open_blobs(self, d_in: int, refs: np.ndarray, d_out: int,
                   hip_stream: Optional[int] = None, ctx: Optional[Context] = None) -> np.ndarray:
        """Per-blob status: 0 ok, 1 MAC mismatch (or < 32 bytes), 2 < 16 bytes."""
        refs = np.ascontiguousarray(refs, AEAD_REF)
        status = np.zeros(max(len(refs), 1), np.uint32)
        c = ctx or _ctx()
        st = _lib.lib().rcdc_aead_open(c.handle, self._kbuf, ctypes.c_void_p(d_in),
                                       refs.ctypes.data, len(refs), ctypes.c_void_p(d_out),
                                       status.ctypes.data, ctypes.c_void_p(hip_stream or 0))
        if st:
            raise status_error(st, _lib.last_error())
        return status[:len(refs)]

    # ---- CryptoKey (aespoly1305.rs:78-135), one blob through HBM -------
    def encrypt_data(self, data: bytes, nonce: Optional[bytes] = None, device: int = 0) -> bytes:
        import torch
        nonce = os.urandom(16) if nonce is None else bytes(nonce)  # :120-121
        n = len(data)
        dev = torch.device("cuda", device)
        src = torch.zeros(n + 4, dtype=torch.uint8)
        src[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8) if n else src[:0]
        d_in = src.to(dev)
        d_out = torch.empty(n + 32, dtype=torch.uint8, device=dev)
        refs = make_refs([0], [n], [0], nonce)
        with torch.cuda.device(dev):
            s = torch.cuda.current_stream(dev).cuda_stream
            self.seal_blobs(d_in.data_ptr(), refs, d_out.data_ptr(), s, _ctx(device))
            torch.cuda.synchronize(dev)
        return d_out.cpu().numpy().tobytes()

    def decrypt_data(self, data: bytes, device: int = 0) -> bytes:
        import torch
        n = len(data)
        if n < 16:  # :89-94
            raise RusticError(ErrorKind.Cryptography,
                              "Data is too short (less than 16 bytes), cannot decrypt.")
        dev = torch.device("cuda", device)
        src = torch.zeros(n + 4, dtype=torch.uint8)
        src[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        d_in = src.to(dev)
        d_out = torch.empty(max(n - 32, 0) + 16, dtype=torch.uint8, device=dev)
        refs = make_refs([0], [n], [0])
        with torch.cuda.device(dev):
            s = torch.cuda.current_stream(dev).cuda_stream
            st = self.open_blobs(d_in.data_ptr(), refs, d_out.data_ptr(), s, _ctx(device))
        if st[0] != 0:  # :97-108
            raise RusticError(ErrorKind.Cryptography, "Data decryption failed, MAC check failed.")
        return d_out[:n - 32].cpu().numpy().tobytes()
