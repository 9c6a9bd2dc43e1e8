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
