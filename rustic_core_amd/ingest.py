"""Device ingest: rustic's backup data path for files already in HBM, end to
end on one GPU -- chunk, blob ids, dedup, compress, seal, verify, pack.

Reference (per file, on the archiver's worker threads, archiver.rs:195):
- ``FileArchiver::backup_reader`` (archiver/file_archiver.rs:138-168): the
  chunker yields chunks, each gets its id ``hash(&chunk)`` (:151);
- ``Packer::add`` / ``add_with_sizelimit`` (blob/packer.rs:304-315): a blob
  whose id the index already has, or that this packer saw, is skipped;
- ``process_data`` (backend/decrypt.rs:566-572): zstd at the repository's
  level (version 2, configfile.rs:182-193), seal (``Key::encrypt_data``),
  and -- extra_verify, the default (configfile.rs:197-199) -- decrypt and
  decode the sealed blob again and compare (``very_data``, decrypt.rs:508-529);
- ``add_raw`` + ``save`` (packer.rs:615-735): sealed blobs appended to the
  pack, the sealed header and its length after them; the pack closes by
  ``PackSizer`` (packer.rs:65-200); ``Indexer::add`` records each pack.

Here one call takes a batch of streams resident in HBM and keeps every byte
there.  The SHA-256 chain of one chunk is serial (a max-size 8 MiB chunk
takes ~0.27 s on one lane), so the pipeline is built around
the long chunks' ids:
  1. chunk every stream (one plan, rcdc_plan_run);
  2. blob ids in two launches on two streams: chunks up to ``long_chunk``
     bytes, and the longer ones (few lanes, the latency floor);
  3. under the long chunks' ids, the long chunks are compressed, sealed
     into a staging area and verified speculatively (they are mostly new:
     a duplicate's work is dropped), while the short chunks -- where the
     duplicates are (zero runs cut at min) -- wait for their ids, are
     deduplicated, and only the first occurrences are compressed, sealed
     and verified;
  4. once the long ids arrive: dedup, then the new blobs in chunk order are
     grouped into packs and copied into place with their sealed headers
     (rcdc_pack_build_raw, add_raw).
No CPU fallback: every step is a device call through the C ABI.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .chunker import ConfigFile, Context
from .compress import check_frames, compress_blobs, make_refs as zstd_refs, zstd_bounds
from .crypto import Key, make_refs as aead_refs
from .device import DevicePlan, sha256_device
from .errors import ErrorKind, RusticError
from .compress import VERIFY_MESSAGE
from .index import IndexPack, index_packs_from_build
from .pack import PackSizer, build_packs, group_blobs, make_blobs, pack_layout


def _void32(ids: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(ids).view(np.dtype((np.void, 32))).ravel()


def first_occurrences(ids: np.ndarray, order: np.ndarray, known) -> np.ndarray:
    """The chunks among `order` (indices in chunk order) that the packer
    would add (packer.rs:304-315): the first occurrence of each id, unless
    the index already has it (`known`, a set of 32-byte ids)."""
    out = np.zeros(len(ids), bool)
    order = np.sort(np.asarray(order, np.int64))
    if not len(order):
        return out
    _, fi = np.unique(_void32(ids[order]), return_index=True)
    cand = order[fi]
    out[cand] = True
    if known:
        for i in cand:
            if bytes(ids[i]) in known:
                out[i] = False
    return out


def _slots(lens, extra: int = 48, align: int = 16):
    """Offsets of slots of (len + extra) bytes, each `align`-aligned."""
    lens = np.asarray(lens, np.int64)
    sz = (lens + extra + align - 1) // align * align
    offs = np.zeros(len(lens), np.int64)
    if len(lens):
        offs[1:] = np.cumsum(sz)[:-1]
    return offs.astype(np.uint64), int(sz.sum())


@dataclass
class IngestResult:
    """What one ``DeviceIngest.ingest`` call produced."""
    packs: object                 # uint8 CUDA tensor: the pack files back to back
    pack_table: np.ndarray        # PACK rows (out_off, blob0, nblobs, size, header_len)
    blobs: np.ndarray             # PACK_BLOB rows of the new blobs, in pack order
    blob_offsets: np.ndarray      # each new blob's offset in its pack
    cuts: list                    # per stream: its cut list
    ids: np.ndarray               # (chunks, 32): every chunk's id, in chunk order
    new: np.ndarray               # bool per chunk: packed here (first occurrence, not indexed)
    chunk_offs: np.ndarray        # arena offset of every chunk
    chunk_lens: np.ndarray
    ms: dict = field(default_factory=dict)

    @property
    def pack_bytes(self) -> int:
        return int(self.pack_table["size"].sum()) if len(self.pack_table) else 0

    def pack_file(self, k: int) -> bytes:
        p = self.pack_table[k]
        o = int(p["out_off"])
        return self.packs[o:o + int(p["size"])].cpu().numpy().tobytes()

    def pack_ids(self) -> List[bytes]:
        """SHA-256 of each pack file (packer.rs:833): the writer's job, which
        reads the bytes anyway; here on the host."""
        import hashlib
        return [hashlib.sha256(self.pack_file(k)).digest() for k in range(len(self.pack_table))]

    def index_packs(self, pack_ids=None, time_: Optional[str] = None) -> List[IndexPack]:
        """IndexPack per pack (Indexer::add's input, packer.rs:784-791)."""
        from .index import rustic_time
        ids = self.pack_ids() if pack_ids is None else pack_ids
        raw = self.blobs.copy()
        raw["len"] = raw["len"] - 32  # index_packs_from_build adds the seal
        return index_packs_from_build(raw, self.pack_table, self.blob_offsets, ids,
                                      time_ or rustic_time())


class DeviceIngest:
    """The backup data path for streams in HBM (see the module doc).

    ``indexed``: ids the repository already holds (the index's ``has``);
    new blob ids are added to it after each call, as the packer's index
    would.  ``extra_verify`` defaults to the config's (true)."""

    def __init__(self, config: ConfigFile, key: Key, device: int = 0,
                 indexed: Optional[set] = None, extra_verify: Optional[bool] = None,
                 long_chunk: int = 2 << 20, current_size: int = 0):
        self.config = config
        self.key = key
        self.device = device
        self.level = config.zstd()
        self.extra_verify = config.extra_verify_() if extra_verify is None else extra_verify
        self.long_chunk = int(long_chunk)
        self.ctx = Context.get(config.poly(), config.chunk_min_size(), config.chunk_size(),
                               config.chunk_max_size(), device=device)
        self.sizer = PackSizer.from_config(config, 0, current_size)
        self.indexed = indexed if indexed is not None else set()
        self._plan = None
        self._layout = None

    # ---- helpers ----------------------------------------------------------
    def _plan_for(self, offs, lens, arena_len):
        key = (tuple(int(x) for x in offs), tuple(int(x) for x in lens), int(arena_len))
        if self._layout != key:
            if self._plan is not None:
                self._plan.close()
            self._plan = DevicePlan(self.ctx, offs, lens, arena_len)
            self._layout = key
        return self._plan

    def _process(self, torch, arena_ptr, sel, c_offs, c_lens, frames, staging, s_off0, stream):
        """compress (level set) + seal chunks `sel` into staging (from byte
        s_off0 on); returns (sealed offsets, sealed lengths, uncompressed
        lengths, end of the staging used).  Synchronous up to the seal."""
        n = len(sel)
        lens = c_lens[sel]
        if self.level is not None:
            f_offs, _ = _slots(zstd_bounds(lens))
            flens = compress_blobs(self.ctx, arena_ptr, zstd_refs(c_offs[sel], lens, f_offs),
                                   frames.data_ptr(), self.level, stream)
            src, src_offs, src_lens = frames.data_ptr(), f_offs, np.asarray(flens, np.uint64)
        else:
            src, src_offs, src_lens = arena_ptr, c_offs[sel], lens
        s_offs, s_total = _slots(src_lens, 32)
        s_offs = s_offs + np.uint64(s_off0)
        nonces = np.frombuffer(os.urandom(16 * n), np.uint8).reshape(n, 16) if n else \
            np.zeros((0, 16), np.uint8)
        self.key.seal_blobs(src, aead_refs(src_offs, src_lens, s_offs, nonces),
                            staging.data_ptr(), stream, self.ctx)
        return s_offs, src_lens + 32, (lens if self.level is not None else
                                       np.zeros(n, np.uint64)), s_off0 + s_total

    def _verify(self, torch, staging, s_offs, s_lens, arena_ptr, c_offs, c_lens, scratch, stream):
        """very_data for a batch: open (MAC) into `scratch`, decode, compare."""
        n = len(s_lens)
        if not n:
            return
        p_offs, _ = _slots(np.asarray(s_lens, np.uint64) - 32, 16)
        st = self.key.open_blobs(staging.data_ptr(), aead_refs(s_offs, s_lens, p_offs),
                                 scratch.data_ptr(), stream, self.ctx)
        bad = np.nonzero(st)[0]
        if not len(bad):
            st = check_frames(self.ctx, scratch.data_ptr(), p_offs, np.asarray(s_lens) - 32,
                              arena_ptr, c_offs, c_lens, stream, stored=self.level is None)
            bad = np.nonzero(st)[0]
        if len(bad):
            raise RusticError(ErrorKind.Verification,
                              f"{VERIFY_MESSAGE} (chunk at arena offset {int(c_offs[bad[0]])})")

    # ---- the batch ----------------------------------------------------------
    def ingest(self, arena, offs, lens) -> IngestResult:
        """Back up the streams [offs[i], offs[i] + lens[i]) of `arena` (a
        uint8 CUDA tensor, 256-byte aligned)."""
        import torch
        dev = arena.device
        t0 = time.perf_counter()
        ms = {}
        s_main = torch.cuda.current_stream(dev)
        s_short, s_long, s_proc = (torch.cuda.Stream(dev) for _ in range(3))
        ptr = arena.data_ptr()
        # 1. chunk
        plan = self._plan_for(offs, lens, arena.numel())
        plan.run(ptr, s_main.cuda_stream)
        cuts = plan.results()
        c_offs, c_lens = [], []
        for o, c in zip(offs, cuts):
            c = np.asarray(c, np.uint64)
            prev = np.concatenate([np.zeros(1, np.uint64), c[:-1]])
            c_offs.append(np.uint64(o) + prev)
            c_lens.append(c - prev)
        c_offs = np.concatenate(c_offs) if c_offs else np.zeros(0, np.uint64)
        c_lens = np.concatenate(c_lens) if c_lens else np.zeros(0, np.uint64)
        n = len(c_lens)
        ms["chunk"] = (time.perf_counter() - t0) * 1e3
        # 2. ids: short and long chunks on two streams, each longest first
        is_long = c_lens > self.long_chunk
        ids_dev = torch.empty((max(n, 1), 32), dtype=torch.uint8, device=dev)
        groups = {}
        for name, mask, st in (("long", is_long, s_long), ("short", ~is_long, s_short)):
            idx = np.nonzero(mask)[0]
            idx = idx[np.argsort(-c_lens[idx].astype(np.int64), kind="stable")]
            refs = torch.from_numpy(np.stack([c_offs[idx].astype(np.int64),
                                              c_lens[idx].astype(np.int64)], 1)
                                    if len(idx) else np.zeros((0, 2), np.int64)).to(dev)
            st.wait_stream(s_main)
            out = torch.empty((max(len(idx), 1), 32), dtype=torch.uint8, device=dev)
            if len(idx):
                sha256_device(self.ctx, arena, refs, out, st.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(st)
            groups[name] = (idx, out, refs, ev)
        s_proc.wait_stream(s_main)
        sp = s_proc.cuda_stream
        seal_off = np.zeros(n, np.uint64)  # offsets relative to the long staging (mod 2^64)
        seal_len = np.zeros(n, np.uint64)
        ulen = np.zeros(n, np.uint64)
        done = np.zeros(n, bool)

        def bound_bytes(sel):
            return int((zstd_bounds(c_lens[sel]) + 64).sum()) + 64

        # 3a. long chunks, speculatively (before their ids); frames are dead
        # once sealed, so the verify opens into them
        t1 = time.perf_counter()
        lidx = np.sort(groups["long"][0])
        frames = torch.empty(bound_bytes(lidx), dtype=torch.uint8, device=dev)
        st_long = torch.empty(bound_bytes(lidx), dtype=torch.uint8, device=dev)
        base = st_long.data_ptr()
        if len(lidx):
            so, sl, ul, _ = self._process(torch, ptr, lidx, c_offs, c_lens, frames, st_long, 0, sp)
            seal_off[lidx], seal_len[lidx], ulen[lidx] = so, sl, ul
            done[lidx] = True
            if self.extra_verify:
                self._verify(torch, st_long, so, sl, ptr, c_offs[lidx], c_lens[lidx], frames, sp)
        ms["long_speculative"] = (time.perf_counter() - t1) * 1e3
        # 3b. short chunks: ids, dedup, first occurrences only
        ids = np.zeros((n, 32), np.uint8)
        sidx, sout, _, sev = groups["short"]
        sev.synchronize()
        ms["short_ids_ready"] = (time.perf_counter() - t0) * 1e3
        if len(sidx):
            ids[sidx] = sout[:len(sidx)].cpu().numpy()
        known = self.indexed
        first = first_occurrences(ids, sidx, known)
        snew = np.nonzero(first & ~is_long)[0]
        t2 = time.perf_counter()
        st_short = None
        if len(snew):
            need = bound_bytes(snew)
            if frames.numel() < need:
                del frames
                frames = torch.empty(need, dtype=torch.uint8, device=dev)
            st_short = torch.empty(need, dtype=torch.uint8, device=dev)
            so, sl, ul, _ = self._process(torch, ptr, snew, c_offs, c_lens, frames, st_short, 0, sp)
            if self.extra_verify:
                self._verify(torch, st_short, so, sl, ptr, c_offs[snew], c_lens[snew], frames, sp)
            # relative to the long staging's base (64-bit wrap-around offsets)
            rel = np.uint64((st_short.data_ptr() - base) % (1 << 64))
            seal_off[snew], seal_len[snew], ulen[snew] = so + rel, sl, ul
            done[snew] = True
        ms["short_new"] = (time.perf_counter() - t2) * 1e3
        del frames
        # 4. long ids, final dedup over the whole batch in chunk order
        lidx_q, lout, _, lev = groups["long"]
        lev.synchronize()
        ms["long_ids_ready"] = (time.perf_counter() - t0) * 1e3
        if len(lidx_q):
            ids[lidx_q] = lout[:len(lidx_q)].cpu().numpy()
        new = first_occurrences(ids, np.arange(n), known)
        assert done[new].all(), "a new blob was not processed"
        nidx = np.nonzero(new)[0]
        t3 = time.perf_counter()
        nb = len(nidx)
        blobs = make_blobs(seal_off[nidx], seal_len[nidx], ids[nidx], np.zeros((nb, 16), np.uint8),
                           uncompressed=ulen[nidx])
        grp = group_blobs([int(x) - 32 for x in seal_len[nidx]], self.sizer,
                          [int(x) for x in ulen[nidx]])
        hn = np.frombuffer(os.urandom(16 * len(grp)), np.uint8).reshape(len(grp), 16) if grp else \
            np.zeros((0, 16), np.uint8)
        packs_t, total = pack_layout(blobs, grp, hn, raw=True)
        packs = torch.empty(max(total, 1) + 64, dtype=torch.uint8, device=dev)
        offs_in_pack = build_packs(self.ctx, self.key._key, base, blobs, packs_t,
                                   packs.data_ptr(), total, sp, raw=True) if nb else \
            np.zeros(0, np.uint32)
        s_proc.synchronize()
        self.indexed.update(map(bytes, ids[nidx]))
        ms["pack"] = (time.perf_counter() - t3) * 1e3
        ms["total"] = (time.perf_counter() - t0) * 1e3
        del st_long, st_short
        return IngestResult(packs, packs_t, blobs, offs_in_pack, cuts, ids, new, c_offs, c_lens, ms)

    def close(self):
        if self._plan is not None:
            self._plan.close()
            self._plan = None
