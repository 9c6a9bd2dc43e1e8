"""Device-resident batches: the measured hot path (rcdc_plan_* in include/rcdc.h).

A batch is a set of independent streams laid out in one device arena (a torch
``uint8`` CUDA tensor, i.e. HIP memory on ROCm).  ``DevicePlan`` fixes the
layout once (work lists, summaries and cut slots live in HBM) and ``run()``
enqueues the scan and resolve kernels on a HIP stream.  torch is only the
allocator / stream provider here; the C ABI sees plain pointers.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .chunker import Context
from .errors import status_error


def align_up(x: int, a: int = 256) -> int:
    return (x + a - 1) // a * a


def pack_offsets(lens: Sequence[int], align: int = 256):
    """Offsets of streams packed back to back (each ``align``-aligned)."""
    offs, o = [], 0
    for n in lens:
        offs.append(o)
        o = align_up(o + int(n), align)
    return np.array(offs, dtype=np.uint64), o + align


class DevicePlan:
    def __init__(self, ctx: Context, offs, lens, arena_len: int):
        self.ctx = ctx
        self.offs = np.ascontiguousarray(offs, dtype=np.uint64)
        self.lens = np.ascontiguousarray(lens, dtype=np.uint64)
        self.n = int(self.lens.size)
        self.arena_len = int(arena_len)
        h = ctypes.c_void_p()
        st = _lib.lib().rcdc_plan_create(ctx.handle, self.offs.ctypes.data,
                                         self.lens.ctypes.data, self.n, self.arena_len,
                                         ctypes.byref(h))
        if st:
            raise status_error(st, _lib.last_error())
        self._h = h
        self.cap = sum(ctx.max_cuts(int(n)) for n in self.lens)

    def info(self) -> dict:
        inf = _lib.PlanInfo()
        st = _lib.lib().rcdc_plan_get_info(self._h, ctypes.byref(inf))
        if st:
            raise status_error(st, _lib.last_error())
        return {k: getattr(inf, k) for k, _ in _lib.PlanInfo._fields_}

    def run(self, d_arena_ptr: int, hip_stream: Optional[int] = None) -> None:
        st = _lib.lib().rcdc_plan_run(self._h, ctypes.c_void_p(d_arena_ptr),
                                      ctypes.c_void_p(hip_stream or 0))
        if st:
            raise status_error(st, _lib.last_error())

    def results(self) -> list:
        cuts = np.zeros(max(self.cap, 1), dtype=np.uint64)
        counts = np.zeros(max(self.n, 1), dtype=np.uint64)
        st = _lib.lib().rcdc_plan_results(self._h, cuts.ctypes.data, self.cap,
                                          counts.ctypes.data)
        if st:
            raise status_error(st, _lib.last_error())
        out, o = [], 0
        for i in range(self.n):
            k = int(counts[i])
            out.append(cuts[o:o + k].copy())
            o += k
        return out

    def device_results(self):
        """(d_cuts_ptr, d_counts_ptr, cut_base[n]) -- raw device pointers."""
        dc, dn = ctypes.c_uint64(0), ctypes.c_uint64(0)
        base = ctypes.POINTER(ctypes.c_uint64)()
        st = _lib.lib().rcdc_plan_device_results(self._h, ctypes.byref(dc), ctypes.byref(dn),
                                                 ctypes.byref(base))
        if st:
            raise status_error(st, _lib.last_error())
        return dc.value, dn.value, np.ctypeslib.as_array(base, shape=(max(self.n, 1),))[:self.n]

    def window(self, stream: int, bound: int, k: int, d_out_ptr: int,
               hip_stream: Optional[int] = None) -> None:
        """Enqueue the crossing window of ``stream``'s cut list into the device
        buffer ``d_out_ptr`` (3 + k u64: count, index and value of the first
        cut >= ``bound``, the first k cuts; ``rcdc_plan_window``)."""
        st = _lib.lib().rcdc_plan_window(self._h, int(stream), int(bound), int(k),
                                         ctypes.c_void_p(d_out_ptr),
                                         ctypes.c_void_p(hip_stream or 0))
        if st:
            raise status_error(st, _lib.last_error())

    def hash(self, d_arena_ptr: int, hip_stream: Optional[int] = None) -> None:
        """Enqueue the SHA-256 blob id of every chunk of the last ``run``
        (``rcdc_plan_hash``; crypto/hasher.rs:17-19, file_archiver.rs:151)."""
        st = _lib.lib().rcdc_plan_hash(self._h, ctypes.c_void_p(d_arena_ptr),
                                       ctypes.c_void_p(hip_stream or 0))
        if st:
            raise status_error(st, _lib.last_error())

    def digests(self) -> list:
        """Per stream, a ``(k, 32)`` uint8 array of chunk digests in cut order."""
        cap = max(self.cap, 1)
        dig = np.zeros((cap, 32), dtype=np.uint8)
        counts = np.zeros(max(self.n, 1), dtype=np.uint64)
        st = _lib.lib().rcdc_plan_digests(self._h, dig.ctypes.data, cap, counts.ctypes.data)
        if st:
            raise status_error(st, _lib.last_error())
        out, o = [], 0
        for i in range(self.n):
            k = int(counts[i])
            out.append(dig[o:o + k].copy())
            o += k
        return out

    def set_pipeline(self, enable: bool) -> None:
        """Overlap run k's resolve with run k + 1's scan (rcdc_plan_set_pipeline)."""
        st = _lib.lib().rcdc_plan_set_pipeline(self._h, 1 if enable else 0)
        if st:
            raise status_error(st, _lib.last_error())

    def flush_next(self) -> None:
        """The next (pipelined) run is the last of the sequence: its chain
        kernels run on the whole chip (rcdc_plan_set_pipeline(plan, 2))."""
        st = _lib.lib().rcdc_plan_set_pipeline(self._h, 2)
        if st:
            raise status_error(st, _lib.last_error())

    def set_timing(self, enable: bool, every: int = 1) -> None:
        """HIP events around the kernels of every ``every``-th run (see
        ``rcdc_plan_set_timing``); ``enable=False`` stops recording."""
        st = _lib.lib().rcdc_plan_set_timing(self._h, int(every) if enable else 0)
        if st:
            raise status_error(st, _lib.last_error())

    def kernel_times(self):
        """(runs, summed scan ms, summed resolve ms) since set_timing(True)."""
        n, a, b = ctypes.c_uint64(0), ctypes.c_double(0), ctypes.c_double(0)
        st = _lib.lib().rcdc_plan_kernel_times(self._h, ctypes.byref(n), ctypes.byref(a),
                                               ctypes.byref(b))
        if st:
            raise status_error(st, _lib.last_error())
        return n.value, a.value, b.value

    WALK_STAT_NAMES = ("rounds", "zones", "chunks", "fix_rounds", "fix_zones", "fix_cuts",
                       "chk_rounds", "chk_zones", "round_bytes", "chk_round_bytes")

    def walk_stats(self, trace: bool = False, check_trace: bool = False):
        """Work counters of the last run's walk path (rcdc_plan_walk_stats):
        a dict, plus the ``(pieces, 4)`` per-piece trace (t0, t1 in 100 MHz
        ticks, rounds, chunks) when ``trace`` (plan built with
        RCDC_WALK_TRACE=1), plus the per-boundary check trace (t0, t1, gap
        rounds, hop entries; row 0 of each stream unused) when
        ``check_trace``."""
        stats = np.zeros(len(self.WALK_STAT_NAMES), dtype=np.uint64)
        pieces = self.info()["walk_pieces"]
        trace = trace or check_trace
        tr = np.zeros((2 * max(pieces, 1), 4), dtype=np.uint64) if trace else None
        st = _lib.lib().rcdc_plan_walk_stats(self._h, stats.ctypes.data,
                                             tr.ctypes.data if trace else None,
                                             tr.size if trace else 0)
        if st:
            raise status_error(st, _lib.last_error())
        d = {k: int(v) for k, v in zip(self.WALK_STAT_NAMES, stats)}
        if check_trace:
            return d, tr[:pieces], tr[pieces:2 * pieces]
        return (d, tr[:pieces]) if trace else d

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().rcdc_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


def hash_many(plans, d_arena_ptrs, hip_stream: Optional[int] = None) -> None:
    """Blob ids of up to 8 plans' last runs in one launch (rcdc_plan_hash_many)."""
    n = len(plans)
    hs = (ctypes.c_void_p * max(n, 1))(*[p._h.value for p in plans])
    ars = (ctypes.c_void_p * max(n, 1))(*[ctypes.c_void_p(a).value for a in d_arena_ptrs])
    st = _lib.lib().rcdc_plan_hash_many(ctypes.cast(hs, ctypes.c_void_p), n,
                                        ctypes.cast(ars, ctypes.c_void_p),
                                        ctypes.c_void_p(hip_stream or 0))
    if st:
        raise status_error(st, _lib.last_error())


def sha256_host_supported() -> bool:
    """rcdc_sha256_host runs on this CPU (AVX-512F/BW)."""
    return _lib.lib().rcdc_sha256_host(None, None, 0, None) == 0


def sha256_host(addrs, lens) -> list:
    """SHA-256 of host buffers (addresses and lengths; pack files,
    packer.rs:832-834) on the calling thread, 16 at a time in AVX-512 lanes
    (rcdc_sha256_host; the GIL is released during the call).  Raises
    RusticError (Unsupported) on a CPU without AVX-512F/BW."""
    n = len(addrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[int(a) for a in addrs])
    ls = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in lens])
    out = ctypes.create_string_buffer(32 * max(n, 1))
    st = _lib.lib().rcdc_sha256_host(ptrs, ls, n, out)
    if st:
        raise status_error(st, _lib.last_error())
    raw = out.raw
    return [raw[32 * i:32 * i + 32] for i in range(n)]


def sha256_device(ctx: Context, arena_tensor, refs, out_tensor=None, stream=None):
    """SHA-256 of chunks ``refs`` (an ``(n, 2)`` int64 CUDA tensor of
    ``(offset, length)`` rows) of a device arena; returns an ``(n, 32)``
    uint8 CUDA tensor (``rcdc_sha256_chunks``)."""
    import torch

    refs = refs.contiguous()
    n = int(refs.shape[0])
    if refs.dtype != torch.int64 or refs.dim() != 2 or refs.shape[1] != 2:
        raise ValueError("refs must be an (n, 2) int64 tensor")
    if out_tensor is None:
        out_tensor = torch.empty((n, 32), dtype=torch.uint8, device=arena_tensor.device)
    if not stream:  # order after torch's producers of arena / refs
        stream = torch.cuda.current_stream(arena_tensor.device).cuda_stream
    st = _lib.lib().rcdc_sha256_chunks(ctx.handle, ctypes.c_void_p(arena_tensor.data_ptr()),
                                       ctypes.c_void_p(refs.data_ptr()), n,
                                       ctypes.c_void_p(out_tensor.data_ptr()),
                                       ctypes.c_void_p(stream or 0))
    if st:
        raise status_error(st, _lib.last_error())
    return out_tensor


def chunk_device(ctx: Context, arena_tensor, offs, lens, stream=None) -> list:
    """One-shot: plan + run + results over a torch CUDA uint8 arena."""
    plan = DevicePlan(ctx, offs, lens, arena_tensor.numel())
    plan.run(arena_tensor.data_ptr(), stream)
    try:
        return plan.results()
    finally:
        plan.close()
