"""Index files for the packs the device builds (the
index half): what ``Indexer::add`` collects and ``Indexer::save`` persists.

Reference:
- ``repofile/indexfile.rs:24-143``: ``IndexFile { supersedes?, packs,
  packs_to_delete (skipped when empty) }``, ``IndexPack { id, blobs, time?,
  size? }`` (``#[skip_serializing_none]``), ``IndexBlob { id, type, offset,
  length, uncompressed_length }`` (``BlobLocation`` flattened; its
  ``uncompressed_length: Option<NonZeroU32>`` has no skip attribute, so an
  uncompressed blob serialises ``"uncompressed_length":null``);
- ``index/indexer.rs:16-22,114-180``: an index file is saved once it holds
  ``MAX_COUNT`` = 50 000 blobs (or after ``MAX_AGE``, a wall-clock rule not
  modelled), and at ``finalize``; ``has`` answers dedup lookups;
- ``blob/packer.rs:784-791``: a written pack's ``IndexPack`` gets its id and
  ``time = Some(now)`` (``size`` stays ``None``);
- ``backend/decrypt.rs:273-290,441-459``: ``save_file`` serialises with
  ``serde_json::to_vec`` (compact, struct field order) and ``encrypt_file``
  prefixes ``2`` + a zstd frame in version-2 repositories before sealing;
  the file id is the SHA-256 of the sealed bytes (``hash_write_full``).

The JSON is host work (kilobytes per pack); the compression and sealing of
the file go through the device (``compress.encode_all``, ``crypto.Key``).
"""
from __future__ import annotations

import datetime
import hashlib
import json
from dataclasses import dataclass, field
from typing import Iterable, List, Optional

import numpy as np

from .errors import ErrorKind, RusticError

MAX_COUNT = 50_000  # indexer.rs:20

_TYPES = {0: "data", 1: "tree"}
_TYPE_IDS = {v: k for k, v in _TYPES.items()}


@dataclass
class IndexBlob:
    """indexfile.rs IndexBlob: id, type, and the flattened BlobLocation."""
    id: bytes
    type: int  # BlobType: 0 data, 1 tree
    offset: int
    length: int
    uncompressed_length: Optional[int] = None

    def to_obj(self) -> dict:
        return {"id": self.id.hex(), "type": _TYPES[self.type], "offset": int(self.offset),
                "length": int(self.length),
                "uncompressed_length": (int(self.uncompressed_length)
                                        if self.uncompressed_length else None)}

    @classmethod
    def from_obj(cls, o: dict) -> "IndexBlob":
        ul = o.get("uncompressed_length")
        if ul == 0:  # NonZeroU32
            raise RusticError(ErrorKind.InvalidInput, "uncompressed_length 0")
        return cls(bytes.fromhex(o["id"]), _TYPE_IDS[o["type"]], int(o["offset"]),
                   int(o["length"]), int(ul) if ul is not None else None)


@dataclass
class IndexPack:
    """indexfile.rs IndexPack (skip_serializing_none: time / size omitted
    when None)."""
    id: bytes
    blobs: List[IndexBlob] = field(default_factory=list)
    time: Optional[str] = None
    size: Optional[int] = None

    def add(self, id_: bytes, tpe: int, offset: int, length: int,
            uncompressed_length: Optional[int] = None) -> None:  # indexfile.rs:86-104
        self.blobs.append(IndexBlob(bytes(id_), int(tpe), int(offset), int(length),
                                    int(uncompressed_length) if uncompressed_length else None))

    def pack_size(self) -> int:
        """indexfile.rs:108-112 -> PackHeaderRef::from_index_pack(..).pack_size()
        (packfile.rs:355-372): blobs + header entries (37 / 41 bytes) + the
        sealing overhead of the header (32) + its u32 length (4)."""
        if self.size is not None:
            return self.size
        return (sum(b.length for b in self.blobs) +
                sum(41 if b.uncompressed_length else 37 for b in self.blobs) + 32 + 4)

    def to_obj(self) -> dict:
        o = {"id": self.id.hex(), "blobs": [b.to_obj() for b in self.blobs]}
        if self.time is not None:
            o["time"] = self.time
        if self.size is not None:
            o["size"] = int(self.size)
        return o

    @classmethod
    def from_obj(cls, o: dict) -> "IndexPack":
        return cls(bytes.fromhex(o["id"]), [IndexBlob.from_obj(b) for b in o.get("blobs") or []],
                   o.get("time"), o.get("size"))


@dataclass
class IndexFile:
    """indexfile.rs IndexFile."""
    packs: List[IndexPack] = field(default_factory=list)
    packs_to_delete: List[IndexPack] = field(default_factory=list)
    supersedes: Optional[List[bytes]] = None

    def add(self, p: IndexPack, delete: bool = False) -> None:  # indexfile.rs:48-54
        (self.packs_to_delete if delete else self.packs).append(p)

    def to_obj(self) -> dict:
        o = {}
        if self.supersedes is not None:
            o["supersedes"] = [s.hex() for s in self.supersedes]
        o["packs"] = [p.to_obj() for p in self.packs]
        if self.packs_to_delete:
            o["packs_to_delete"] = [p.to_obj() for p in self.packs_to_delete]
        return o

    def to_json(self) -> bytes:
        """serde_json::to_vec: compact, fields in struct order."""
        return json.dumps(self.to_obj(), separators=(",", ":")).encode()

    @classmethod
    def from_json(cls, data: bytes) -> "IndexFile":
        o = json.loads(data)
        sup = o.get("supersedes")
        return cls([IndexPack.from_obj(p) for p in o.get("packs") or []],
                   [IndexPack.from_obj(p) for p in o.get("packs_to_delete") or []],
                   [bytes.fromhex(s) for s in sup] if sup is not None else None)


def rustic_time(t: Optional[datetime.datetime] = None) -> str:
    """RusticTime's Timestamp form (repofile.rs:131-139): RFC 3339 with the
    local offset, nanosecond digits as jiff prints them (trailing zeros
    dropped)."""
    t = (t or datetime.datetime.now(datetime.timezone.utc)).astimezone()
    frac = f"{t.microsecond:06d}000".rstrip("0")
    off = t.strftime("%z")
    return t.strftime("%Y-%m-%dT%H:%M:%S") + (("." + frac) if frac else "") + \
        off[:3] + ":" + off[3:]


def index_packs_from_build(blobs: np.ndarray, packs: np.ndarray, offsets: np.ndarray,
                           pack_ids: Iterable[bytes], time: Optional[str] = None
                           ) -> List[IndexPack]:
    """IndexPack per built pack (rcdc_pack_build outputs): each blob's
    offset in its pack, sealed length (len + 32), type, id and raw length;
    the pack id (SHA-256 of the pack file, packer.rs:833) from the caller."""
    out = []
    for p, pid in zip(packs, pack_ids):
        ip = IndexPack(bytes(pid), time=time)
        b0, n = int(p["blob0"]), int(p["nblobs"])
        for i in range(b0, b0 + n):
            b = blobs[i]
            ip.add(bytes(b["id"]), int(b["type"]), int(offsets[i]), int(b["len"]) + 32,
                   int(b["uncompressed_len"]) or None)
        out.append(ip)
    return out


class Indexer:
    """index/indexer.rs:30-180: collects IndexPacks into IndexFiles; `save`
    hands a file to `save_file` (a callable taking the IndexFile, returning
    its id) once MAX_COUNT blobs are held, and at `finalize`."""

    def __init__(self, save_file, indexed: Optional[set] = None):
        self._save_file = save_file
        self.file = IndexFile()
        self.count = 0
        self.indexed = indexed  # None: no dedup tracking (Indexer::new_unindexed)
        self.saved: List[bytes] = []

    def add(self, pack: IndexPack, delete: bool = False) -> None:  # :151-180
        self.count += len(pack.blobs)
        if self.indexed is not None:
            for b in pack.blobs:
                self.indexed.add(b.id)
        self.file.add(pack, delete)
        if self.count >= MAX_COUNT:
            self.save()
            self.file = IndexFile()
            self.count = 0

    def save(self) -> None:  # :114-119
        if self.file.packs or self.file.packs_to_delete:
            self.saved.append(self._save_file(self.file))

    def finalize(self) -> None:
        self.save()

    def has(self, blob_id: bytes) -> bool:  # :187-191
        return self.indexed is not None and bytes(blob_id) in self.indexed


def encrypt_file(key, data: bytes, version: int = 2, level: int = 0, nonce=None,
                 device: int = 0) -> bytes:
    """DecryptBackend::encrypt_file (decrypt.rs:441-459): version 2 seals
    2 || zstd(data), version 1 the data as is; both on the device."""
    from .compress import encode_all
    payload = bytes([2]) + encode_all(data, level, device) if version >= 2 else bytes(data)
    return key.encrypt_data(payload, nonce, device)


def save_index_file(key, index: IndexFile, version: int = 2, level: int = 0, nonce=None,
                    device: int = 0):
    """save_file (decrypt.rs:273-290): (IndexId = SHA-256 of the sealed
    bytes, sealed bytes)."""
    sealed = encrypt_file(key, index.to_json(), version, level, nonce, device)
    return hashlib.sha256(sealed).digest(), sealed
