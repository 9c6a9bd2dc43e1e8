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
from .device import DevicePlan, sha256_device, sha256_host, sha256_host_supported
from .errors import ErrorKind, RusticError
from .compress import VERIFY_MESSAGE
from .index import IndexPack, index_packs_from_build
from .pack import (PACK_BLOB, PackSizer, build_packs_multi, copy_ranges, group_blobs_open,
                   make_blobs, pack_layout)

_SRC_LONG, _SRC_SHORT, _SRC_CARRY = 0, 1, 2  # blobs["pad"]: the sealed blob's buffer


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
    blobs: np.ndarray             # PACK_BLOB rows of the packed blobs, in pack order (the
                                  # open pack's carried blobs first; in_off is relative to
                                  # the sealed-blob buffer `pad`, dead after the call)
    blob_offsets: np.ndarray      # each packed blob's offset in its pack
    cuts: list                    # per stream: its cut list
    ids: np.ndarray               # (chunks, 32): every chunk's id, in chunk order
    new: np.ndarray               # bool per chunk: added to the packer (first occurrence, not
                                  # indexed) -- in a pack here or in the still open pack
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


@dataclass
class _Pending:
    """A batch between DeviceIngest.begin and .end."""
    arena: object
    ptr: int
    t0: float
    ms: dict
    s_proc: object
    groups: dict
    cuts: list
    c_offs: np.ndarray
    c_lens: np.ndarray
    is_long: np.ndarray
    seal_off: np.ndarray
    seal_len: np.ndarray
    seal_src: np.ndarray
    ulen: np.ndarray
    done: np.ndarray
    frames: object = None
    st_long: object = None

    def bound_bytes(self, sel) -> int:
        return int((zstd_bounds(self.c_lens[sel]) + 64).sum()) + 64


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
        # two sets of (short ids, long ids, processing) streams, alternating
        # per begin(): a batch in flight next to the previous one gets its own
        # queues (its long ids do not wait behind the previous batch's), and
        # the caching allocator reuses each set's blocks (it pools per stream)
        self._streams = None
        self._nbegin = 0
        # the open pack (blobs added, pack not yet saved): its sealed blobs in
        # a device buffer of their own, PACK_BLOB rows with pad = _SRC_CARRY
        self._carry = None
        self._carry_blobs = np.zeros(0, PACK_BLOB)

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
    def ingest(self, arena, offs, lens, finalize: bool = False) -> IngestResult:
        """Back up the streams [offs[i], offs[i] + lens[i]) of `arena` (a
        uint8 CUDA tensor, 256-byte aligned).  The packer stays open between
        calls, as rustic's one Packer per backup (packer.rs:659-671): the
        packs should_save closes are returned, the blobs of the still open
        pack stay on the device for the next call (``finalize`` closes it
        too, as ``finalize()`` does alone).  Work on `arena` is ordered after
        the caller's current stream.  ``end(begin(...))``."""
        return self.end(self.begin(arena, offs, lens), finalize)

    def _stream_set(self, torch, dev):
        if self._streams is None:
            self._streams = [tuple(torch.cuda.Stream(dev) for _ in range(3)) for _ in range(2)]
        st = self._streams[self._nbegin % 2]
        self._nbegin += 1
        return st

    def begin(self, arena, offs, lens, plan: Optional[DevicePlan] = None,
              host_ids=None) -> "_Pending":
        """First half of ``ingest``: chunk, launch every chunk's blob id and
        compress + seal + verify the long chunks speculatively.  The long ids
        (the SHA-256 latency floor) are still running on return, so a caller
        streaming batches runs ``begin(k + 1)`` before ``end(k)`` and the
        floors of consecutive batches overlap (HostIngest).  Until ``end`` the
        arena must stay unchanged; ``end`` calls must come in ``begin``
        order (dedup and the open pack are sequential).

        ``host_ids(chunk_arena_offsets, chunk_lengths)``: when the caller
        still holds the bytes in host memory it may compute the long chunks'
        ids there (a callable returning a future of an ``(n, 32)`` uint8
        array): one host core hashes a chunk ~75x faster than one device lane
        (~2.4 GB/s vs 64 B per 2 us), so for the last batch of a stream of
        batches, whose long-id chain is not hidden under later batches, the
        host is the shorter path."""
        import torch
        dev = arena.device
        t0 = time.perf_counter()
        ms = {}
        s_main = torch.cuda.current_stream(dev)
        s_short, s_long, s_proc = self._stream_set(torch, dev)
        ptr = arena.data_ptr()
        # 1. chunk (a plan built for this layout beforehand, or the cached one)
        if plan is None:
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
        groups = {}
        for name, mask, st in (("long", is_long, s_long), ("short", ~is_long, s_short)):
            idx = np.nonzero(mask)[0]
            idx = idx[np.argsort(-c_lens[idx].astype(np.int64), kind="stable")]
            if name == "long" and host_ids is not None:
                groups[name] = (idx, host_ids(c_offs[idx], c_lens[idx]), None, None)
                continue
            st.wait_stream(s_main)
            with torch.cuda.stream(st):  # the buffers belong to the stream using them
                refs = torch.from_numpy(np.stack([c_offs[idx].astype(np.int64),
                                                  c_lens[idx].astype(np.int64)], 1)
                                        if len(idx) else np.zeros((0, 2), np.int64)).to(dev)
                out = torch.empty((max(len(idx), 1), 32), dtype=torch.uint8, device=dev)
            if len(idx):
                sha256_device(self.ctx, arena, refs, out, st.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(st)
            groups[name] = (idx, out, refs, ev)
        s_proc.wait_stream(s_main)
        p = _Pending(arena=arena, ptr=ptr, t0=t0, ms=ms, s_proc=s_proc, groups=groups, cuts=cuts,
                     c_offs=c_offs, c_lens=c_lens, is_long=is_long,
                     seal_off=np.zeros(n, np.uint64), seal_len=np.zeros(n, np.uint64),
                     seal_src=np.zeros(n, np.uint32), ulen=np.zeros(n, np.uint64),
                     done=np.zeros(n, bool))
        # 3a. long chunks, speculatively (before their ids); frames are dead
        # once sealed, so the verify opens into them.  Every buffer the
        # kernels on s_proc use is allocated on s_proc (the caching allocator
        # then never hands its memory to another stream while they run).
        # Sealed blobs: source 0 = the long staging, 1 = the short staging,
        # 2 = the open pack carried over from the last call (_SRC_*).
        t1 = time.perf_counter()
        lidx = np.sort(groups["long"][0])
        with torch.cuda.stream(s_proc):
            p.frames = torch.empty(p.bound_bytes(lidx), dtype=torch.uint8, device=dev)
            p.st_long = torch.empty(p.bound_bytes(lidx), dtype=torch.uint8, device=dev)
        if len(lidx):
            sp = s_proc.cuda_stream
            so, sl, ul, _ = self._process(torch, ptr, lidx, c_offs, c_lens, p.frames, p.st_long, 0,
                                          sp)
            p.seal_off[lidx], p.seal_len[lidx], p.ulen[lidx] = so, sl, ul
            p.seal_src[lidx] = _SRC_LONG
            p.done[lidx] = True
            if self.extra_verify:
                self._verify(torch, p.st_long, so, sl, ptr, c_offs[lidx], c_lens[lidx], p.frames,
                             sp)
        ms["long_speculative"] = (time.perf_counter() - t1) * 1e3
        return p

    def end(self, p: "_Pending", finalize: bool = False) -> IngestResult:
        """Second half of ``ingest`` (see ``begin``): dedup the short chunks
        on their ids and process the first occurrences, wait for the long
        ids, dedup the whole batch in chunk order and pack."""
        import torch
        dev = p.arena.device
        ms, t0, ptr = p.ms, p.t0, p.ptr
        s_proc, sp = p.s_proc, p.s_proc.cuda_stream
        c_offs, c_lens, is_long = p.c_offs, p.c_lens, p.is_long
        n = len(c_lens)
        # 3b. short chunks: ids, dedup, first occurrences only
        ids = np.zeros((n, 32), np.uint8)
        sidx, sout, _, sev = p.groups["short"]
        sev.synchronize()
        ms["short_ids_ready"] = (time.perf_counter() - t0) * 1e3
        if len(sidx):
            ids[sidx] = sout[:len(sidx)].cpu().numpy()
        known = self.indexed
        first = first_occurrences(ids, sidx, known)
        snew = np.nonzero(first & ~is_long)[0]
        t2 = time.perf_counter()
        st_short = None
        frames = p.frames
        p.frames = None
        if len(snew):
            need = p.bound_bytes(snew)
            with torch.cuda.stream(s_proc):
                if frames.numel() < need:
                    del frames
                    frames = torch.empty(need, dtype=torch.uint8, device=dev)
                st_short = torch.empty(need, dtype=torch.uint8, device=dev)
            so, sl, ul, _ = self._process(torch, ptr, snew, c_offs, c_lens, frames, st_short, 0, sp)
            if self.extra_verify:
                self._verify(torch, st_short, so, sl, ptr, c_offs[snew], c_lens[snew], frames, sp)
            p.seal_off[snew], p.seal_len[snew], p.ulen[snew] = so, sl, ul
            p.seal_src[snew] = _SRC_SHORT
            p.done[snew] = True
        ms["short_new"] = (time.perf_counter() - t2) * 1e3
        del frames
        # 4. long ids, final dedup over the whole batch in chunk order
        lidx_q, lout, _, lev = p.groups["long"]
        if lev is None:  # ids computed on the host (begin's host_ids)
            got = lout.result()
            ms["long_ids_ready"] = (time.perf_counter() - t0) * 1e3
            if len(lidx_q):
                ids[lidx_q] = got
        else:
            lev.synchronize()
            ms["long_ids_ready"] = (time.perf_counter() - t0) * 1e3
            if len(lidx_q):
                ids[lidx_q] = lout[:len(lidx_q)].cpu().numpy()
        new = first_occurrences(ids, np.arange(n), known)
        assert p.done[new].all(), "a new blob was not processed"
        nidx = np.nonzero(new)[0]
        t3 = time.perf_counter()
        nb = len(nidx)
        blobs_new = make_blobs(p.seal_off[nidx], p.seal_len[nidx], ids[nidx],
                               np.zeros((nb, 16), np.uint8), uncompressed=p.ulen[nidx])
        blobs_new["pad"] = p.seal_src[nidx]
        st_long = p.st_long
        srcs = [st_long.data_ptr(), (st_short if st_short is not None else st_long).data_ptr(),
                self._carry.data_ptr() if self._carry is not None else st_long.data_ptr()]
        res = self._pack(torch, np.concatenate([self._carry_blobs, blobs_new]), srcs, finalize, sp,
                         s_proc, dev)
        # indexed only once packed (or carried in the open pack): a failed
        # _pack must not make later calls dedup these blobs away
        self.indexed.update(map(bytes, ids[nidx]))
        ms["pack"] = (time.perf_counter() - t3) * 1e3
        ms["total"] = (time.perf_counter() - t0) * 1e3
        p.st_long = None
        del st_long, st_short
        packs, packs_t, blobs, offs_in_pack = res
        return IngestResult(packs, packs_t, blobs, offs_in_pack, p.cuts, ids, new, c_offs, c_lens,
                            ms)

    def finalize(self) -> IngestResult:
        """Close the open pack (Packer::finalize, packer.rs:385-398): its
        blobs, carried from earlier calls, become the last pack."""
        import torch
        dev = torch.device("cuda", self.device)
        s_proc = torch.cuda.Stream(dev)
        s_proc.wait_stream(torch.cuda.current_stream(dev))
        srcs = [self._carry.data_ptr()] * 3 if self._carry is not None else [0, 0, 0]
        t0 = time.perf_counter()
        packs, packs_t, blobs, offs_in_pack = self._pack(torch, self._carry_blobs, srcs, True,
                                                         s_proc.cuda_stream, s_proc, dev)
        z = np.zeros(0, np.uint64)
        return IngestResult(packs, packs_t, blobs, offs_in_pack, [], np.zeros((0, 32), np.uint8),
                            np.zeros(0, bool), z, z, {"pack": (time.perf_counter() - t0) * 1e3})

    @property
    def open_blobs(self) -> int:
        """Blobs of the open pack (added, not yet in a pack file)."""
        return len(self._carry_blobs)

    def _pack(self, torch, blobs, srcs, finalize, sp, s_proc, dev):
        """Group `blobs` (the open pack's first, then this call's new ones, in
        chunk order) as the packer does, build the packs should_save closes
        (rcdc_pack_build_raw_multi over the sealed blobs' buffers) and move the
        open pack's blobs into a new carry buffer (rcdc_copy_ranges)."""
        grp, open_from = group_blobs_open([int(x) - 32 for x in blobs["len"]], self.sizer,
                                          [int(x) for x in blobs["uncompressed_len"]], finalize)
        closed = blobs[:open_from]
        hn = np.frombuffer(os.urandom(16 * len(grp)), np.uint8).reshape(len(grp), 16) if grp else \
            np.zeros((0, 16), np.uint8)
        packs_t, total = pack_layout(closed, grp, hn, raw=True)
        with torch.cuda.stream(s_proc):
            packs = torch.empty(max(total, 1) + 64, dtype=torch.uint8, device=dev)
        offs_in_pack = build_packs_multi(self.ctx, self.key._key, srcs, closed, packs_t,
                                         packs.data_ptr(), total, sp) if len(grp) else \
            np.zeros(0, np.uint32)
        rest = blobs[open_from:].copy()
        carry = None
        if len(rest):
            lens = rest["len"].astype(np.uint64)
            dst = np.zeros(len(rest), np.uint64)
            dst[1:] = np.cumsum((lens + 15) // 16 * 16)[:-1]
            with torch.cuda.stream(s_proc):
                carry = torch.empty(int(dst[-1] + lens[-1]) + 64, dtype=torch.uint8, device=dev)
            copy_ranges(self.ctx, srcs, rest["pad"], rest["in_off"], lens, dst, carry.data_ptr(),
                        sp)
            rest["in_off"] = dst
            rest["pad"] = _SRC_CARRY
        s_proc.synchronize()
        self._carry, self._carry_blobs = carry, rest
        return packs, packs_t, closed, offs_in_pack

    def close(self):
        if self._plan is not None:
            self._plan.close()
            self._plan = None


# ---- files in host memory -> packs and pack ids in host memory -------------
@dataclass
class HostIngestResult:
    """What ``HostIngest.run`` produced: every pack file in host memory (one
    pinned buffer, packs back to back), their ids, and per batch the device
    results (cuts, chunk ids, dedup decisions)."""
    packs_host: object            # uint8 CPU tensor (pinned): pack files back to back
    pack_offs: np.ndarray         # each pack's offset in packs_host
    pack_sizes: np.ndarray
    pack_ids: List[bytes]         # SHA-256 of each pack file (packer.rs:832-834)
    batches: List[IngestResult]   # per batch (their .packs device tensors dropped)
    batch_files: List[List[int]]  # the files of each batch
    seconds: float                # wall time: first H2D issued .. last pack id computed
    h2d_bytes: int
    d2h_bytes: int
    ms: dict = field(default_factory=dict)

    def pack_file(self, k: int) -> bytes:
        o = int(self.pack_offs[k])
        return self.packs_host[o:o + int(self.pack_sizes[k])].numpy().tobytes()


def plan_batches(sizes, first: int, middle: int, last: int,
                 taper: bool = True) -> List[List[int]]:
    """Whole files in order into batches of about ``first`` bytes, then
    ``middle``, and a tail ending in one of about ``last`` (``taper``: a
    halving tail middle/2, middle/4, ... down to ``last``): a small first
    batch starts the device early, a shrinking tail shortens the drain (each
    batch's packs reach the host hash threads about one batch after its copy;
    the pack ids of a middle batch arriving last would hold them ~0.25 s)."""
    total = int(sum(sizes))
    tail = [last]
    if taper:
        b = middle // 2
        while b > last and total >= first + middle + sum(tail) + b:
            tail.insert(len(tail) - 1, b)
            b //= 2
    rest = total - first - sum(tail)
    m = max(-(-rest // middle), 0)
    targets = [first] + [-(-rest // m)] * m + tail if m else [first] + tail
    ends = np.cumsum(targets)  # a batch closes where the running total would pass its end
    out, cur, acc, t = [], [], 0, 0
    for i, n in enumerate(sizes):
        if cur and t < len(ends) - 1 and acc + n > ends[t]:
            out.append(cur)
            cur, t = [], t + 1
        cur.append(i)
        acc += int(n)
    if cur:
        out.append(cur)
    return out


class HostIngest:
    """The backup data path from files in host memory to pack files and pack
    ids in host memory, on one GPU.

    Reference: ``FileArchiver::backup_reader`` reads each file and chunks it
    (archiver/file_archiver.rs:144-160), ``Packer`` packs the new blobs
    (blob/packer.rs:260-275, 615-735), hashes each finished pack file for its
    id (``hash_reader``, packer.rs:832-834) and hands it to the backend.

    Pipeline over batches of whole files (``plan_batches``), three device
    arena slots:
      - H2D of batch k + 2 (one copy stream) while the device works on k, k + 1;
      - ``DeviceIngest.begin(k)`` (chunk, launch ids, long chunks
        speculatively) before ``end(k - 1)`` (dedup, short chunks, packs), so
        the SHA-256 latency floors of consecutive batches overlap;
      - D2H of each batch's packs (a second copy stream, the other PCIe
        direction) into one pinned host buffer;
      - pack ids on ``hash_threads`` host threads (hashlib: OpenSSL SHA-256,
        the GIL released), each pack as soon as its batch's copy is done.
    The packer stays open across batches (one pack sequence, as one Packer
    per backup) and the last batch finalizes it.

    The process should give HIP more hardware queues than its default 4
    (environment GPU_MAX_HW_QUEUES, e.g. 16, before the first HIP call): HIP
    maps streams onto them round robin, and a kernel queued behind a
    multi-GiB copy on a shared queue waits for that copy (the short ids of
    one batch waited ~0.3 s behind the next batch's H2D with 4 queues)."""

    def __init__(self, config: ConfigFile, key: Key, device: int = 0,
                 indexed: Optional[set] = None, extra_verify: Optional[bool] = None,
                 hash_threads: Optional[int] = None, first_batch: int = 2 << 30,
                 batch: int = 8 << 30, last_batch: int = 1 << 30,
                 pack_ratio: float = 0.8):
        self.ingest = DeviceIngest(config, key, device, indexed, extra_verify)
        self.device = device
        if hash_threads is None:  # the job's CPUs (the main thread mostly waits on the GPU)
            try:
                hash_threads = len(os.sched_getaffinity(0))
            except AttributeError:  # pragma: no cover
                hash_threads = 8
            omp = os.environ.get("OMP_NUM_THREADS", "")
            if omp.isdigit() and int(omp) > 0:
                hash_threads = min(hash_threads, int(omp))
        self.hash_threads = int(hash_threads)
        self.first_batch, self.batch, self.last_batch = int(first_batch), int(batch), int(last_batch)
        self.pack_ratio = float(pack_ratio)  # initial pinned pack buffer / input bytes
        self.d2h_group = 512 << 20  # pack bytes per copy-back event
        # the first and last batches' long-chunk ids on host threads from the
        # files (their device chains are not hidden under other batches:
        # ~0.27 s per 8 MiB chunk)
        self.host_edge_ids = True
        self.host_tail_ids = 3  # the last batches whose long ids the host computes
        # pack ids of all but the last hashlib_tail batches 16 packs at a time
        # in AVX-512 lanes (rcdc_sha256_host: ~2x a core's SHA extensions per
        # core); the last batches' packs one per thread (hashlib), whose
        # latency (~16 ms per 40 MB pack, not ~16x that) the run's end waits on
        self.multi_buffer_ids = sha256_host_supported()
        self.hashlib_tail = 2  # the last batches whose pack ids go one per thread
        # batches before those hashed 8 packs per call (half the lanes, half the
        # latency); 0: measured best (groups of 8 left a larger backlog)
        self.mb_half_batches = 0

    def run(self, files) -> HostIngestResult:
        """`files`: 1-D uint8 CPU tensors (pinned for full-rate copies)."""
        import hashlib
        import threading
        from concurrent.futures import ThreadPoolExecutor

        import torch
        from .device import pack_offsets
        dev = torch.device("cuda", self.device)
        sizes = [int(f.numel()) for f in files]
        batches = plan_batches(sizes, self.first_batch, self.batch, self.last_batch)
        layouts = [pack_offsets([sizes[i] for i in b]) for b in batches]
        slot_len = max(a for _, a in layouts)
        arenas = [torch.empty(slot_len, dtype=torch.uint8, device=dev)
                  for _ in range(min(3, len(batches)))]
        total_in = sum(sizes)
        host = torch.empty(int(total_in * self.pack_ratio) + (64 << 20), dtype=torch.uint8,
                           pin_memory=True)
        s_h2d, s_d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        ev_h2d = [None] * len(batches)
        pool = ThreadPoolExecutor(max_workers=self.hash_threads)
        # one thread waits for the copy-back events (in order) and hands each
        # landed group to the hash threads: a hash thread never blocks on one
        waiter = ThreadPoolExecutor(max_workers=1)
        lock = threading.Lock()
        ids_out, offs_out, sizes_out, futs, keep = [], [], [], [], []
        state = {"host_off": 0, "d2h": 0, "host": host}
        ms = {"begin": 0.0, "end": 0.0, "handoff": 0.0}  # host wall ms per step

        def h2d(k):
            offs, _ = layouts[k]
            a = arenas[k % len(arenas)]
            with torch.cuda.stream(s_h2d):
                for i, o in zip(batches[k], offs):
                    a[int(o):int(o) + sizes[i]].copy_(files[i], non_blocking=True)
                ev_h2d[k] = torch.cuda.Event()
                ev_h2d[k].record(s_h2d)

        hstat = {"busy_s": 0.0, "first": None, "last": 0.0}

        def hash_pack(buf, o, n, slot):
            a = time.perf_counter()
            d = hashlib.sha256(memoryview(buf[o:o + n].numpy())).digest()
            b = time.perf_counter()
            with lock:
                ids_out[slot] = d
                hstat["busy_s"] += b - a
                hstat["first"] = a if hstat["first"] is None else min(hstat["first"], a)
                hstat["last"] = max(hstat["last"], b)

        def hash_group(buf, grp, j0, base_addr):
            # one call, up to 16 packs side by side (GIL released inside)
            a = time.perf_counter()
            ds = sha256_host([base_addr + o for o, _ in grp], [n for _, n in grp])
            b = time.perf_counter()
            with lock:
                for j, d in enumerate(ds):
                    ids_out[j0 + j] = d
                hstat["busy_s"] += b - a
                hstat["first"] = a if hstat["first"] is None else min(hstat["first"], a)
                hstat["last"] = max(hstat["last"], b)

        def handoff(res, k):
            # the packs of one batch: D2H into the pinned buffer, then hashed
            t = time.perf_counter()
            total = res.pack_bytes
            if total:
                o0 = state["host_off"]
                if o0 + total > state["host"].numel():  # (rare) a larger buffer
                    s_d2h.synchronize()
                    big = torch.empty(int((o0 + total) * 1.25), dtype=torch.uint8,
                                      pin_memory=True)
                    big[:o0].copy_(state["host"][:o0])
                    state["host"] = big
                buf = state["host"]
                rows = [(int(p["out_off"]), int(p["size"])) for p in res.pack_table]
                base = len(ids_out)
                ids_out.extend([None] * len(rows))
                for o, n in rows:
                    offs_out.append(o0 + o)
                    sizes_out.append(n)
                # the copy back in groups of packs of >= d2h_group bytes, one
                # event each: hashing starts with the first group, not after
                # the whole batch
                g0 = 0
                mb = self.multi_buffer_ids and k < len(batches) - self.hashlib_tail
                mb_n = 8 if k >= len(batches) - self.hashlib_tail - self.mb_half_batches else 16
                with torch.cuda.stream(s_d2h):
                    s_d2h.wait_stream(torch.cuda.current_stream(dev))
                    while g0 < len(rows):
                        g1, gb = g0, 0
                        while g1 < len(rows) and (g1 == g0 or (g1 - g0 < mb_n if mb else
                                                               gb < self.d2h_group)):
                            gb += rows[g1][1]
                            g1 += 1
                        a, e = rows[g0][0], rows[g1 - 1][0] + rows[g1 - 1][1]
                        buf[o0 + a:o0 + e].copy_(res.packs[a:e], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(s_d2h)

                        def job(ev=ev, grp=rows[g0:g1], j0=base + g0, buf=buf, mb=mb):
                            ev.synchronize()
                            if mb:
                                return [pool.submit(hash_group, buf, [(o0 + o, n) for o, n in grp],
                                                    j0, buf.data_ptr())]
                            return [pool.submit(hash_pack, buf, o0 + o, n, j0 + j)
                                    for j, (o, n) in enumerate(grp)]
                        futs.append(waiter.submit(job))
                        g0 = g1
                    ev_all = torch.cuda.Event()
                    ev_all.record(s_d2h)
                keep.append((res.packs, ev_all))
                state["host_off"] = o0 + total
                state["d2h"] += total
            res.packs = None
            ms["handoff"] += (time.perf_counter() - t) * 1e3

        plans = []
        id_pool = ThreadPoolExecutor(max_workers=self.hash_threads)
        try:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            # the batches' chunking plans first (work lists and cut buffers:
            # building one allocates device memory and uploads synchronously, so
            # none is built inside the pipeline or behind the queued copies)
            plans += [DevicePlan(self.ingest.ctx, offs, [sizes[i] for i in b], slot_len)
                     for b, (offs, _) in zip(batches, layouts)]
            ms["plans"] = (time.perf_counter() - t0) * 1e3
            for k in range(min(len(arenas), len(batches))):
                h2d(k)
            results, pending = [], None

            def host_ids_for(k):
                # the batch's long-chunk ids from the files in host memory
                offs_k = np.asarray(layouts[k][0], np.uint64)
                files_k = batches[k]

                def one(a, n):
                    j = int(np.searchsorted(offs_k, a, side="right")) - 1
                    o = int(a - offs_k[j])
                    f = files[files_k[j]]
                    return hashlib.sha256(memoryview(f[o:o + int(n)].numpy())).digest()

                def run(c_offs_sel, c_lens_sel):
                    futs_ = [id_pool.submit(one, int(a), int(n)) for a, n in zip(c_offs_sel, c_lens_sel)]

                    class _All:
                        def result(self_):
                            out = np.zeros((len(futs_), 32), np.uint8)
                            for i, f_ in enumerate(futs_):
                                out[i] = np.frombuffer(f_.result(), np.uint8)
                            return out
                    return _All()
                return run

            for k in range(len(batches)):
                torch.cuda.current_stream(dev).wait_event(ev_h2d[k])
                offs, _ = layouts[k]
                t = time.perf_counter()
                # the first and last batches' long-chunk ids on the host: the
                # first batch's packs then reach the hash threads sooner (they are
                # idle until then), the last one's follow the last copy at once
                edge = (k == 0 or k >= len(batches) - self.host_tail_ids) and len(batches) > 1
                p = self.ingest.begin(arenas[k % len(arenas)], offs, [sizes[i] for i in batches[k]],
                                      plan=plans[k],
                                      host_ids=host_ids_for(k) if edge and self.host_edge_ids else None)
                ms["begin"] += (time.perf_counter() - t) * 1e3
                ms[f"begin{k}"] = (time.perf_counter() - t) * 1e3
                if pending is not None:
                    t = time.perf_counter()
                    r = self.ingest.end(pending)
                    ms["end"] += (time.perf_counter() - t) * 1e3
                    ms[f"end{k - 1}"] = (time.perf_counter() - t) * 1e3
                    ms[f"at{k - 1}"] = (time.perf_counter() - t0) * 1e3
                    handoff(r, k - 1)
                    results.append(r)
                    # the slot of batch k - 1 is free: batch k + 2 goes there
                    if k + 2 < len(batches):
                        h2d(k + 2)
                pending = p
            t = time.perf_counter()
            r = self.ingest.end(pending, finalize=True)
            ms["end"] += (time.perf_counter() - t) * 1e3
            handoff(r, len(batches) - 1)
            results.append(r)
            ms["last_end"] = (time.perf_counter() - t0) * 1e3
            for f in futs:  # the per-batch waiters, then their pack jobs
                for g in f.result():
                    g.result()
            seconds = time.perf_counter() - t0
            # pack-id hashing: thread-seconds spent, and its window
            ms["hash_thread_s"] = round(hstat["busy_s"], 3)
            if hstat["first"] is not None:
                ms["hash_first_ms"] = (hstat["first"] - t0) * 1e3
                ms["hash_last_ms"] = (hstat["last"] - t0) * 1e3
            for r in results:  # per-phase times of each batch
                ms.setdefault("batch_ms", []).append({k: round(v, 1) for k, v in r.ms.items()})
        finally:
            # on any exit: the hash and wait threads stop, the plans' device
            # buffers and the arena slots are released
            waiter.shutdown()
            pool.shutdown()
            id_pool.shutdown()
            for pl in plans:
                pl.close()
            keep.clear()
            arenas.clear()
        return HostIngestResult(state["host"], np.asarray(offs_out, np.int64),
                                np.asarray(sizes_out, np.int64), list(ids_out), results, batches,
                                seconds, total_in, state["d2h"], ms)

    def close(self):
        self.ingest.close()
