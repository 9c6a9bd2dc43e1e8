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

    Slices may be EMPTY (a_r == b_r == total): rounding the share up to a
    multiple of min leaves the trailing ranks nothing when the stream is
    short for the world (8 MiB + 1 byte over 8 ranks at min 512 KiB: ranks
    6 and 7).  Callers keep such ranks in every collective of the stitch
    (chunk_long_stream_sharded, SlicedStream.stitch).
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


def window_len(min_size: int, max_size: int) -> int:
    """Head cuts a crossing window carries: the true chain enters slice r at
    x < a_r + max, and the chain from a_r has at most max / min cuts below
    that (every chunk but the last is >= min)."""
    return max_size // min_size + 2


NONE = np.int64(-1)  # UINT64_MAX as the int64 the collectives move


def host_window(cuts_rel, bound_rel: int, k: int) -> np.ndarray:
    """The crossing window of a host cut list (relative to its chain start):
    [n, j, c[j], c[0..k)] with j the first cut >= bound_rel -- the same words
    rcdc_plan_window writes on the device (include/rcdc.h)."""
    c = np.asarray(cuts_rel, dtype=np.int64)
    n = len(c)
    j = int(np.searchsorted(c, bound_rel))
    out = np.full(3 + k, NONE, dtype=np.int64)
    out[0], out[1] = n, j
    if j < n:
        out[2] = c[j]
    m = min(k, n)
    out[3:3 + m] = c[:m]
    return out


def stitch_windows(bounds, entries, wins, k: int):
    """Walk the ranks in order over their crossing windows.  wins[r] is rank
    r's window of the chain that starts at entries[r] (relative cuts, list
    truncated after its first cut >= b_r).  Returns (per rank (i0, j): its
    true cuts are list[i0 .. j], or None for none; first rank that could not
    be merged and the true entry it needs, or None)."""
    out = []
    x = 0  # true chain position entering slice r
    for r, (a, b, _) in enumerate(bounds):
        if x >= b or a >= b:
            out.append(None)
            continue
        w = np.asarray(wins[r], dtype=np.int64)
        n, j = int(w[0]), int(w[1])
        if x == entries[r]:
            i0 = 0
        else:
            head = w[3:3 + min(k, n)] + entries[r]
            hit = np.flatnonzero(head == x)
            if not len(hit):
                return out, (r, x)
            i0 = int(hit[0]) + 1
        out.append((i0, j))
        if j < n:
            x = int(w[2]) + entries[r]
    return out, None


def _all_gather_windows(win, world: int, group=None):
    """One fixed-size all_gather of every rank's window (3 + k words):
    torch tensors on the device over RCCL, on the host over gloo."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [win.cpu().numpy() if hasattr(win, "cpu") else np.asarray(win)]
    t = win if isinstance(win, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(win))
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        t = t.cpu()
    elif dist.get_backend(group) != "gloo" and not t.is_cuda:
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return list(out.cpu().numpy().reshape(world, -1))


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
    fixed-size crossing windows (window_len + 3 words per rank, never the
    lists) lets every rank walk the chain in order; a rank whose window does
    not contain the true entry cut re-chunks from that entry (another round;
    every rank tracks the entries, so they are not exchanged).  Returns this
    rank's true cuts (absolute; rank 0 starts at 0).
    """
    import torch.distributed as dist
    bounds = slice_bounds(total, world, min_size, max_size)
    a, b, _ = bounds[rank]
    k = window_len(min_size, max_size)
    entries = [bb[0] for bb in bounds]
    mine = np.asarray(chunk_from(a), dtype=np.uint64) if a < b else np.zeros(0, np.uint64)
    distributed = world > 1 and dist.is_available() and dist.is_initialized()
    if world > 1 and not distributed:
        raise RuntimeError("chunk_long_stream_sharded: world > 1 needs torch.distributed")
    while True:
        win = host_window(mine.astype(np.int64) - entries[rank], b - entries[rank], k)
        wins = _all_gather_windows(win, world, group)
        spans, todo = stitch_windows(bounds, entries, wins, k)
        if todo is None:
            sp = spans[rank]
            return mine[sp[0]:sp[1] + 1] if sp is not None else np.zeros(0, np.uint64)
        r, x = todo
        entries[r] = x
        if r == rank:
            mine = np.asarray(chunk_from(x), dtype=np.uint64)


class SlicedStream:
    """The device side of one stream sliced over ranks (bench.py C5): this
    rank's slice [a, b) plus its halo up to e sits at offset 0 of `arena`; a
    plan over the whole extent chunks it from a.  `step()` runs the plan and
    stitches: rcdc_plan_window writes the crossing window into a device
    buffer, one all_gather of those windows (RCCL on the device; gloo
    through the host) and the host walk of the ranks decide which part of
    the device cut list is true.  The lists stay on their ranks; a rank whose
    window misses the true entry re-chunks from it with a fresh plan (host
    list).  At world 1 the chain from 0 is the truth: nothing to stitch."""

    def __init__(self, ctx, arena, plan, total: int, rank: int, world: int,
                 min_size: int, max_size: int, stream=None, group=None):
        import torch
        self.ctx, self.arena, self.plan = ctx, arena, plan
        self.total, self.rank, self.world, self.group = total, rank, world, group
        self.bounds = slice_bounds(total, world, min_size, max_size)
        self.a, self.b, self.e = self.bounds[rank]
        self.k = window_len(min_size, max_size)
        self.stream = stream
        self.win = torch.empty(3 + self.k, dtype=torch.int64, device=arena.device)
        self.chunk_from = device_chunk_from(ctx, arena, self.a, self.b, self.e, total,
                                            stream=stream)
        self.last = None
        self.stitch_s, self.nstitch = 0.0, 0  # world > 1: plan end -> stitch result

    def step(self):
        self.plan.run(self.arena.data_ptr(), self.stream)
        if self.world == 1:
            self.last = self.stitch()
            return self.last
        # the stitch waits for the plan anyway (its window, then the gather's
        # host copy): wait here first, so the time from the plan's end to the
        # stitch result (window + all_gather + .cpu() + host walk) is measured
        import time

        import torch
        if self.arena.is_cuda:
            torch.cuda.synchronize(self.arena.device)
        t1 = time.perf_counter()
        self.last = self.stitch()
        self.stitch_s += time.perf_counter() - t1
        self.nstitch += 1
        return self.last

    def stitch(self):
        """(source, i0, j): this rank's true cuts are source[i0 .. j] --
        source "plan" (the device list, relative to a) or a host array of
        absolute cuts (a re-chunked entry).  j None: to the list's end."""
        import torch
        empty = self.a >= self.b
        if self.world == 1:
            return ("plan", 0, None) if not empty else (np.zeros(0, np.uint64), 0, -1)
        entries = [bb[0] for bb in self.bounds]
        mine = None  # host list once this rank has re-chunked
        while True:
            if empty:
                # an empty slice (slice_bounds: trailing ranks of a short
                # stream) owns no cut, but every all_gather of the stitch
                # needs every rank: it sends a window of n = 0 each round
                win = host_window(np.zeros(0, np.int64), 0, self.k)
            elif mine is None:
                self.plan.window(0, self.b - self.a, self.k, self.win.data_ptr(), self.stream)
                if self.stream:
                    torch.cuda.current_stream(self.arena.device).wait_stream(
                        torch.cuda.ExternalStream(self.stream, device=self.arena.device))
                win = self.win
            else:
                win = host_window(mine.astype(np.int64) - entries[self.rank],
                                  self.b - entries[self.rank], self.k)
            wins = _all_gather_windows(win, self.world, self.group)
            if not empty and int(wins[self.rank][0]) == -1:  # the walk needs host completion
                mine = self.plan.results()[0] + np.uint64(self.a)
                if self.e < self.total:
                    mine = mine[:int(np.searchsorted(mine, self.b)) + 1]
                continue
            if any(int(w[0]) == -1 for w in wins):
                continue  # another rank completes on the host and sends again
            spans, todo = stitch_windows(self.bounds, entries, wins, self.k)
            if todo is None:
                sp = spans[self.rank]
                if sp is None:
                    return (np.zeros(0, np.uint64), 0, -1)
                return ("plan" if mine is None else mine, sp[0], sp[1])
            r, x = todo
            entries[r] = x
            if r == self.rank:
                mine = np.asarray(self.chunk_from(x), dtype=np.uint64)

    def cuts(self, res=None) -> np.ndarray:
        """This rank's true cuts (absolute) of the last step's result."""
        src, i0, j = res if res is not None else self.last
        if isinstance(src, str):
            c = self.plan.results()[0] + np.uint64(self.a)
            if self.e < self.total:
                c = c[:int(np.searchsorted(c, self.b)) + 1]
        else:
            c = src
        return c[i0:] if j is None else c[i0:j + 1]


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
