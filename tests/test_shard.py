"""CPU: multi-GPU sharding logic with world_size-2 gloo.

The per-rank chunk function here is the oracle (the test's stand-in for the
device path, which needs a GPU); what is under test is the LPT assignment
and the gather of cut lists back into input order.
"""
import os
import socket

import numpy as np
import pytest

from rustic_core_amd.shard import assign_lpt, local_streams


def test_lpt_balanced_and_complete():
    rng = np.random.default_rng(1)
    lens = [int(x) for x in rng.integers(1, 1 << 30, 500)]
    for world in (1, 2, 3, 8):
        a = assign_lpt(lens, world)
        flat = sorted(i for r in a for i in r)
        assert flat == list(range(len(lens)))
        loads = [sum(lens[i] for i in r) for r in a]
        # LPT bound: max load <= optimum * 4/3, optimum >= max(mean, largest)
        opt_lb = max(sum(lens) / world, max(lens))
        assert max(loads) <= opt_lb * 4 / 3 + 1


def test_lpt_deterministic_and_rank_local():
    lens = [5, 5, 5, 9, 1, 0, 7]
    a = assign_lpt(lens, 3)
    assert a == assign_lpt(list(lens), 3)
    assert [local_streams(lens, r, 3) for r in range(3)] == a
    assert assign_lpt([], 4) == [[], [], [], []]
    with pytest.raises(ValueError):
        assign_lpt(lens, 0)


def _streams():
    rng = np.random.default_rng(7)
    lens = [0, 100, 70000, 300000, 5000, 190000, 64, 250000, 12345]
    data = []
    for i, n in enumerate(lens):
        if i % 3 == 2:
            data.append(np.zeros(n, np.uint8))
        else:
            data.append(rng.integers(0, 256, n, dtype=np.uint8))
    return lens, data


PARAMS = dict(min_size=4096, avg=16384, max_size=65536)


def _worker(rank, world, port, errfile):
    import torch.distributed as dist
    from oracle import oracle
    from rustic_core_amd.shard import chunk_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lens, data = _streams()

        def chunk_local(idx):
            return {i: oracle.chunk_cuts(data[i], oracle.DEFAULT_POLY, **PARAMS) for i in idx}

        got = chunk_sharded(lens, rank, world, chunk_local)
        for i in range(len(lens)):
            want = oracle.chunk_cuts(data[i], oracle.DEFAULT_POLY, **PARAMS)
            assert np.array_equal(got[i], want), i
        dist.barrier()
    except Exception as e:  # pragma: no cover - reported through the file
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {e!r}\n")
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_chunk_sharded_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    err = str(tmp_path / "err.txt")
    mp.spawn(_worker, args=(2, _free_port(), err), nprocs=2, join=True)
    assert not os.path.exists(err)


# ------------------------------------------------- one long stream over ranks
LPARAMS = dict(min_size=4096, avg=16384, max_size=65536)


def _long_data(kind):
    rng = np.random.default_rng(21)
    n = 1_000_003
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "phase_zeros":   # true chain out of phase with the slice starts
        a = np.zeros(n, np.uint8)
        a[:777] = rng.integers(0, 256, 777, dtype=np.uint8)
        return a
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8)
    out = np.zeros(n, np.uint8)
    i = 0
    while i < n:
        k = int(rng.integers(1000, 60000))
        if rng.random() < 0.5:
            out[i:i + k] = rng.integers(0, 256, len(out[i:i + k]), dtype=np.uint8)
        i += k
    return out


def _long_worker(rank, world, port, errfile, kind):
    import torch.distributed as dist
    from oracle import oracle
    from rustic_core_amd.shard import chunk_long_stream_sharded, slice_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = _long_data(kind)
        total = len(data)
        bounds = slice_bounds(total, world, LPARAMS["min_size"], LPARAMS["max_size"])
        a, b, e = bounds[rank]
        local = data[a:e]  # this rank's bytes only: slice + halo

        def chunk_from(s):
            cuts = oracle.chunk_cuts(local[s - a:], oracle.DEFAULT_POLY, **LPARAMS) + s
            if e < total:  # truncate after the crossing cut (the rest sees a fake end)
                k = int(np.searchsorted(cuts, b))
                cuts = cuts[:k + 1]
                assert len(cuts) and int(cuts[-1]) >= b
            return cuts

        mine = chunk_long_stream_sharded(total, rank, world, LPARAMS["min_size"],
                                         LPARAMS["max_size"], chunk_from)
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        got = np.concatenate([np.asarray(p, np.uint64) for p in parts])
        want = oracle.chunk_cuts(data, oracle.DEFAULT_POLY, **LPARAMS)
        assert np.array_equal(got, want), (kind, len(got), len(want))
        dist.barrier()
    except Exception as ex:  # pragma: no cover
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {ex!r}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [(k, w) for w in (2, 3) for k in
                                        ("zeros", "phase_zeros", "random", "mixed")] +
                         [("phase_zeros", 8), ("mixed", 8)])
def test_long_stream_sharded_gloo(tmp_path, kind, world):
    import torch.multiprocessing as mp
    err = str(tmp_path / "err.txt")
    mp.spawn(_long_worker, args=(world, _free_port(), err, kind), nprocs=world, join=True)
    assert not os.path.exists(err)


def test_slice_bounds():
    from rustic_core_amd.shard import slice_bounds
    b = slice_bounds(10_000_000, 4, 4096, 65536)
    assert b[0][0] == 0 and b[-1][1] == 10_000_000
    for (a, bb, e), nxt in zip(b, b[1:] + [(10_000_000, 0, 0)]):
        assert a % 4096 == 0 and bb == nxt[0] and e == min(bb + 65536 + 64, 10_000_000)
    # a short stream leaves the trailing slices empty (documented)
    total = (8 << 20) + 1
    b = slice_bounds(total, 8, 512 << 10, 8 << 20)
    assert [r for r, (a, bb, _) in enumerate(b) if a >= bb] == [6, 7]
    assert b[5][1] == total and all(x == (total, total, total) for x in b[6:])


class _HostPlan:
    """Stand-in for DevicePlan on the CPU: the oracle chunks the rank's extent
    [a, e) as one stream; window() writes the crossing window into the tensor
    whose data_ptr SlicedStream passes (what rcdc_plan_window does on the
    device)."""

    def __init__(self, local, params, win_tensor):
        self.local, self.params, self.win_tensor = local, params, win_tensor
        self.cuts = None

    def run(self, ptr, stream):
        from oracle import oracle
        self.cuts = oracle.chunk_cuts(self.local, oracle.DEFAULT_POLY, *self.params)

    def window(self, stream_i, bound, k, ptr, stream):
        import torch
        from rustic_core_amd.shard import host_window
        assert ptr == self.win_tensor.data_ptr()
        self.win_tensor.copy_(torch.from_numpy(host_window(self.cuts.astype(np.int64), bound, k)))

    def results(self):
        return [self.cuts]


def _sliced_host_worker(rank, world, port, errfile, total, kind):
    import torch
    import torch.distributed as dist
    from oracle import oracle
    from rustic_core_amd.shard import SlicedStream, slice_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = (512 << 10, 1 << 20, 8 << 20)
        rng = np.random.default_rng(31)
        data = (np.zeros(total, np.uint8) if kind == "zeros"
                else rng.integers(0, 256, total, dtype=np.uint8))
        a, b, e = slice_bounds(total, world, params[0], params[2])[rank]
        arena = torch.zeros(e - a + 256, dtype=torch.uint8)

        class _Ctx:  # SlicedStream builds its re-chunk closure lazily
            pass
        ss = SlicedStream(_Ctx(), arena, None, total, rank, world, params[0], params[2])
        ss.plan = _HostPlan(data[a:e], params, ss.win)

        def chunk_from(s):
            cuts = oracle.chunk_cuts(data[s:e], oracle.DEFAULT_POLY, *params) + np.uint64(s)
            if e < total:
                cuts = cuts[:int(np.searchsorted(cuts, b)) + 1]
            return cuts
        ss.chunk_from = chunk_from
        mine = ss.cuts(ss.step())
        parts = [None] * world
        dist.all_gather_object(parts, np.asarray(mine, np.uint64))
        got = np.concatenate(parts)
        want = oracle.chunk_cuts(data, oracle.DEFAULT_POLY, *params)
        assert np.array_equal(got, want), (len(got), len(want))
        dist.barrier()
    except Exception as ex:  # pragma: no cover
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {ex!r}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["zeros", "random"])
def test_sliced_stream_empty_slices_gloo_world8(tmp_path, kind):
    """SlicedStream.stitch with empty trailing slices (8 MiB + 1 over 8 ranks
    at the default parameters: ranks 6 and 7 own nothing) -- they still take
    part in every all_gather, so the stitch returns instead of deadlocking."""
    import torch.multiprocessing as mp
    err = str(tmp_path / "err.txt")
    mp.spawn(_sliced_host_worker, args=(8, _free_port(), err, (8 << 20) + 1, kind), nprocs=8,
             join=True)
    assert not os.path.exists(err)


def test_stitch_windows_rules():
    """The host walk over crossing windows: merge at a head cut, the merged
    rank's crossing feeds the next, and the first rank whose window misses
    the true entry is reported."""
    from rustic_core_amd.shard import host_window, stitch_windows
    k = 4
    bounds = [(0, 100, 150), (100, 200, 250), (200, 300, 300)]
    entries = [0, 100, 200]
    l0 = np.array([40, 80, 120], np.int64)          # crossing 120
    l1 = np.array([20, 60, 110, 150], np.int64)     # abs 120 160 210 250: crossing 210
    l2 = np.array([10, 50, 100], np.int64)          # abs 210 250 300
    w = [host_window(l0, 100, k), host_window(l1, 100, k), host_window(l2, 100, k)]
    spans, todo = stitch_windows(bounds, entries, w, k)
    assert todo is None and spans == [(0, 2), (1, 2), (1, 2)]
    # rank 2's chain misses 210: it must re-chunk from there
    l2b = np.array([15, 55, 100], np.int64)
    spans, todo = stitch_windows(bounds, entries, w[:2] + [host_window(l2b, 100, k)], k)
    assert todo == (2, 210) and spans == [(0, 2), (1, 2)]
    # the chain jumps over a whole slice
    bounds = [(0, 100, 300), (100, 120, 300), (120, 300, 300)]
    w = [host_window(np.array([40, 150, 300], np.int64), 100, k),
         host_window(np.array([30], np.int64), 20, k),
         host_window(np.array([30, 180], np.int64), 180, k)]
    spans, todo = stitch_windows(bounds, [0, 100, 120], w, k)
    assert todo is None and spans == [(0, 1), None, (1, 1)]


def test_long_stream_single_rank_no_process_group():
    """world 1 needs no process group (bench.py C5 at N=1)."""
    from oracle import oracle
    from rustic_core_amd.shard import chunk_long_stream_sharded
    data = _long_data("mixed")
    cuts = chunk_long_stream_sharded(
        len(data), 0, 1, LPARAMS["min_size"], LPARAMS["max_size"],
        lambda s: oracle.chunk_cuts(data[s:], oracle.DEFAULT_POLY, **LPARAMS) + s)
    assert np.array_equal(cuts, oracle.chunk_cuts(data, oracle.DEFAULT_POLY, **LPARAMS))


# ------------------------------------- the device path over ranks (GPU, gloo)
def _device_long_worker(rank, world, port, errfile, kind, params, sliced=False):
    """Rank r holds only its slice + halo on cuda:0 and chunks it with the real
    device plan (shard.device_chunk_from); the cross-rank stitch runs over
    gloo (several ranks share the one GPU of the test box)."""
    import torch
    import torch.distributed as dist
    from oracle import oracle
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.shard import chunk_long_stream_sharded, device_chunk_from, slice_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mn, avg, mx = params
        data = _long_data(kind) if mn < 65536 else _long_data_big(kind)
        total = len(data)
        a, b, e = slice_bounds(total, world, mn, mx)[rank]
        torch.cuda.set_device(0)
        arena = torch.zeros(e - a + 256, dtype=torch.uint8, device="cuda:0")
        arena[:e - a] = torch.from_numpy(np.ascontiguousarray(data[a:e])).to("cuda:0")
        ctx = Context.get(oracle.DEFAULT_POLY, mn, avg, mx, device=0)
        if sliced:  # bench.py C5's path: device windows, fixed-size gather
            from rustic_core_amd.device import DevicePlan
            from rustic_core_amd.shard import SlicedStream
            plan = DevicePlan(ctx, np.zeros(1, np.uint64), np.array([e - a], np.uint64),
                              int(arena.numel()))
            ss = SlicedStream(ctx, arena, plan, total, rank, world, mn, mx,
                              stream=torch.cuda.Stream("cuda:0").cuda_stream)
            ss.step()
            mine = ss.cuts(ss.step())  # twice: the plan and its window are reused
            plan.close()
        else:
            mine = chunk_long_stream_sharded(total, rank, world, mn, mx,
                                             device_chunk_from(ctx, arena, a, b, e, total))
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        got = np.concatenate([np.asarray(p, np.uint64) for p in parts])
        want = oracle.chunk_cuts(data, oracle.DEFAULT_POLY, mn, avg, mx)
        assert np.array_equal(got, want), (kind, len(got), len(want))
        dist.barrier()
    except Exception as ex:  # pragma: no cover
        with open(errfile, "a") as f:
            f.write(f"rank {rank}: {ex!r}\n")
        raise
    finally:
        dist.destroy_process_group()


def _long_data_big(kind):
    """40 MiB + 3 for the default parameters (min 512 KiB)."""
    rng = np.random.default_rng(22)
    n = 40 * (1 << 20) + 3
    if kind == "short_random":  # 8 MiB + 1: over 8 ranks, ranks 6 and 7 get empty slices
        return rng.integers(0, 256, (8 << 20) + 1, dtype=np.uint8)
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "phase_zeros":
        a = np.zeros(n, np.uint8)
        a[:123457] = rng.integers(0, 256, 123457, dtype=np.uint8)
        return a
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8)
    out = np.zeros(n, np.uint8)
    i = 0
    while i < n:
        k = int(rng.integers(64 << 10, 4 << 20))
        if rng.random() < 0.5:
            out[i:i + k] = rng.integers(0, 256, len(out[i:i + k]), dtype=np.uint8)
        i += k
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["zeros", "phase_zeros", "random", "mixed"])
@pytest.mark.parametrize("params", [(4096, 16384, 65536), (512 << 10, 1 << 20, 8 << 20)],
                         ids=["small", "default"])
def test_long_stream_sharded_device_gloo(tmp_path, kind, params):
    import torch.multiprocessing as mp
    err = str(tmp_path / "err.txt")
    mp.spawn(_device_long_worker, args=(2, _free_port(), err, kind, params), nprocs=2, join=True)
    assert not os.path.exists(err)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["zeros", "phase_zeros", "random", "mixed"])
@pytest.mark.parametrize("world", [2, 4])
def test_sliced_stream_device_gloo(tmp_path, kind, world):
    """shard.SlicedStream (bench.py C5): every rank's crossing window from
    rcdc_plan_window, one fixed-size all_gather, re-chunks where a window
    misses the true entry; the concatenated true lists equal the oracle's."""
    import torch.multiprocessing as mp
    err = str(tmp_path / "err.txt")
    mp.spawn(_device_long_worker, args=(world, _free_port(), err, kind, (4096, 16384, 65536),
                                        True), nprocs=world, join=True)
    assert not os.path.exists(err)


@pytest.mark.gpu
def test_sliced_stream_device_gloo_empty_slices(tmp_path):
    """The device C5 path at world 8 with empty trailing slices (8 MiB + 1 at
    the default parameters): ranks 6 and 7 send n = 0 windows and the stitch
    returns on every rank."""
    import torch.multiprocessing as mp
    err = str(tmp_path / "err.txt")
    mp.spawn(_device_long_worker, args=(8, _free_port(), err, "short_random",
                                        (512 << 10, 1 << 20, 8 << 20), True), nprocs=8, join=True)
    assert not os.path.exists(err)
