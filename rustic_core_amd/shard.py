"""Multi-GPU sharding of independent streams.

rustic chunks every file independently, one ChunkIter per file on pariter
workers (crates/core/src/archiver.rs:195, file_archiver.rs:144-160), so the
path shards by file with no data exchange: each rank (one process per GPU,
torch.distributed) chunks the files assigned to it and only the cut lists
travel, once, to the rank that hands them on (the packer side).

  assign_lpt(lens, world)          largest-first onto the least-loaded rank
  local_streams(lens, rank, world) this rank's stream indices (deterministic)
  gather_cuts(local, rank, world)  all ranks' {index: cuts} -> input order
"""
from __future__ import annotations

import heapq
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np


def assign_lpt(lens: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of streams to `world` ranks.

    Streams sorted by length (descending, index breaks ties) each go to the
    rank with the fewest bytes so far (lowest rank breaks ties).  The result
    is a pure function of (lens, world), so every rank computes the same
    assignment without communication.  Max load <= 4/3 of optimal.
    """
    if world < 1:
        raise ValueError("world size must be >= 1")
    order = sorted(range(len(lens)), key=lambda i: (-int(lens[i]), i))
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + int(lens[i]), r))
    for r in range(world):
        out[r].sort()
    return out


def local_streams(lens: Sequence[int], rank: int, world: int) -> List[int]:
    return assign_lpt(lens, world)[rank]


def gather_cuts(local: Dict[int, np.ndarray], n_streams: int, group=None,
                dst: Optional[int] = None) -> Optional[List[np.ndarray]]:
    """Collect every rank's {stream index: cut offsets} into input order.

    One all_gather_object (or gather_object to `dst`) of the per-rank
    results; this is the only collective of the sharded path and it moves
    the outputs (8 B per cut), never the stream bytes.  Returns the full
    list on every rank (dst None) or on `dst` only.
    """
    import torch.distributed as dist
    payload = {int(k): np.asarray(v, dtype=np.uint64) for k, v in local.items()}
    world = dist.get_world_size(group)
    if dst is None:
        parts: list = [None] * world
        dist.all_gather_object(parts, payload, group=group)
    else:
        parts = [None] * world if dist.get_rank(group) == dst else None
        dist.gather_object(payload, parts, dst=dst, group=group)
        if parts is None:
            return None
    out: List[Optional[np.ndarray]] = [None] * n_streams
    for p in parts:
        for k, v in p.items():
            if out[k] is not None:
                raise RuntimeError(f"stream {k} chunked by two ranks")
            out[k] = v
    missing = [i for i, v in enumerate(out) if v is None]
    if missing:
        raise RuntimeError(f"streams {missing[:8]} not chunked by any rank")
    return out  # type: ignore[return-value]


def chunk_sharded(lens: Sequence[int], rank: int, world: int,
                  chunk_local: Callable[[List[int]], Dict[int, np.ndarray]],
                  group=None) -> List[np.ndarray]:
    """Chunk all streams over `world` ranks: this rank runs `chunk_local` on
    its LPT share (the device path: rustic_core_amd.device.chunk_device over
    an arena holding those streams) and all ranks receive every cut list."""
    mine = local_streams(lens, rank, world)
    local = chunk_local(mine)
    if set(local) != set(mine):
        raise RuntimeError("chunk_local returned a different stream set")
    return gather_cuts(local, len(lens), group=group)


# ---------------------------------------------------------------- one long stream
def slice_bounds(total: int, world: int, min_size: int, max_size: int):
    """Split one stream of `total` bytes into `world` slices [a_r, b_r) whose
    starts are multiples of min (long zero runs then stay in phase, every
    chunk there being exactly min), plus each rank's readable extent
    [a_r, e_r): the slice and a halo of max + 64 bytes from the next slice,
    enough for the chain that starts before b_r to reach its crossing cut
    exactly (no hop from s < b_r looks past s + max + 63).
    """
    per = -(-total // world)
    per = -(-per // min_size) * min_size
    out = []
    for r in range(world):
        a = min(r * per, total)
        b = min(a + per, total)
        e = min(b + max_size + 64, total)
        out.append((a, b, e))
    return out


def _stitch_lists(bounds, lists, total):
    """Walk the ranks in order.  lists[r] = (entry, cuts): cuts of the chain
    that starts at `entry` (absolute), ending with its first cut >= b_r (or
    total).  Returns (true cut lists per rank, first rank that could not be
    merged and the true entry it needs, or None)."""
    true = []
    x = 0  # true chain position entering slice r
    for r, (a, b, _) in enumerate(bounds):
        entry, cuts = lists[r]
        if x >= b or a >= b:
            true.append(np.zeros(0, np.uint64))
            continue
        cuts = np.asarray(cuts, dtype=np.uint64)
        if x == entry:
            keep = cuts
        else:
            i = int(np.searchsorted(cuts, x))
            if i < len(cuts) and int(cuts[i]) == x:
                keep = cuts[i + 1:]
            else:
                return true, (r, x)
        true.append(keep)
        if len(keep):
            x = int(keep[-1])
    return true, None


def chunk_long_stream_sharded(total: int, rank: int, world: int, min_size: int,
                              max_size: int, chunk_from: Callable[[int], np.ndarray],
                              group=None) -> np.ndarray:
    """Chunk ONE stream of `total` bytes split over `world` ranks
    (SURVEY.md 8(e), C5).  Rank r owns bytes [a_r, e_r) (slice_bounds);
    `chunk_from(s)` must return the absolute cuts of the chain that starts at
    absolute position s, computed on this rank's bytes and truncated after
    the first cut >= b_r (the device path: a plan over arena[s - a_r, e_r -
    a_r) as an independent stream; its cuts up to the crossing are exact
    because the halo covers s + max + 63).

    Every rank chunks its slice speculatively from a_r; one all_gather of
    the cut lists lets every rank walk the chain in order; a rank whose list
    does not contain the true entry cut re-chunks from that entry (another
    round).  Returns this rank's true cuts (absolute; rank 0 starts at 0).
    """
    import torch.distributed as dist
    bounds = slice_bounds(total, world, min_size, max_size)
    a, b, _ = bounds[rank]
    entry = a
    mine = np.asarray(chunk_from(a), dtype=np.uint64) if a < b else np.zeros(0, np.uint64)
    distributed = world > 1 and dist.is_available() and dist.is_initialized()
    if world > 1 and not distributed:
        raise RuntimeError("chunk_long_stream_sharded: world > 1 needs torch.distributed")
    while True:
        parts: list = [None] * world
        if distributed:
            dist.all_gather_object(parts, (entry, mine), group=group)
        else:
            parts[0] = (entry, mine)
        true, todo = _stitch_lists(bounds, parts, total)
        if todo is None:
            return true[rank]
        r, x = todo
        if r == rank:
            entry = x
            mine = np.asarray(chunk_from(x), dtype=np.uint64)


def device_chunk_from(ctx, arena, a: int, b: int, e: int, total: int, first_plan=None,
                      stream: Optional[int] = None) -> Callable[[int], np.ndarray]:
    """The device `chunk_from` of chunk_long_stream_sharded for rank slice
    [a, b) with readable extent [a, e): `arena` (a CUDA uint8 tensor) holds
    stream bytes [a, e) at offset 0.  The chain from s is a fresh plan over
    arena[s - a, e - a) as an independent stream (a stream starting at s is
    exactly the chain with a cut at s), or `first_plan`'s last run for
    s == a; cuts are truncated after the first one >= b (beyond it the halo's
    end looks like EOF)."""
    from .device import DevicePlan

    def chunk_from(s: int) -> np.ndarray:
        if s == a and first_plan is not None:
            cuts = first_plan.results()[0] + np.uint64(a)
        else:
            p = DevicePlan(ctx, np.array([s - a], np.uint64), np.array([e - s], np.uint64),
                           int(arena.numel()))
            try:
                p.run(arena.data_ptr(), stream)
                cuts = p.results()[0] + np.uint64(s)
            finally:
                p.close()
        if e < total:
            cuts = cuts[:int(np.searchsorted(cuts, b)) + 1]
        return cuts

    return chunk_from
