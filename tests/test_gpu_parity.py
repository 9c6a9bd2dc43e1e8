"""Device parity: librcdc (HIP, gfx950) vs the CPU oracle and the reference's
golden snapshots.  Bit-exact cut offsets are the bar (integer work).

Every case runs through the C ABI (rcdc_plan_*, rcdc_chunk_batch,
rcdc_stream_feed); the oracle is only the checker.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_snapshots.json")
MiB = 1 << 20
KiB = 1 << 10


def _torch():
    import torch
    return torch


def _device_cuts(ctx, bufs, offsets=None, align=256):
    """Chunk host buffers via a device-resident plan; returns per-buffer cuts."""
    torch = _torch()
    from rustic_core_amd.device import DevicePlan, pack_offsets
    lens = [len(b) for b in bufs]
    if offsets is None:
        offs, arena_len = pack_offsets(lens, align)
    else:
        offs = np.array(offsets, dtype=np.uint64)
        arena_len = int(max([o + n for o, n in zip(offsets, lens)] + [0])) + 256
    host = np.zeros(arena_len, dtype=np.uint8)
    for o, b in zip(offs, bufs):
        host[int(o):int(o) + len(b)] = np.frombuffer(bytes(b), np.uint8) if not isinstance(
            b, np.ndarray) else b
    dev = torch.from_numpy(host).to("cuda:0")
    plan = DevicePlan(ctx, offs, lens, arena_len)
    plan.run(dev.data_ptr())
    out = plan.results()
    plan.close()
    return out


def _ctx(min_size, avg, max_size, poly=oracle.DEFAULT_POLY):
    from rustic_core_amd.chunker import Context
    return Context.get(poly, min_size, avg, max_size, device=0)


# ---------------------------------------------------------------- golden pins
def test_chunk_random_snapshot(gpu_ctx):
    """rabin.rs:341-358 + chunk_random.snap: all 29 (len, sha256) exact."""
    from rustic_core_amd import ChunkIter, ConfigFile
    g = json.load(open(GOLDEN))["rabin_chunk_random"]
    data = oracle.stdrng_bytes(g["seed"], g["size"]).tobytes()
    cfg = ConfigFile.new(2, int(g["poly"], 16))
    chunks = [(len(c), hashlib.sha256(c).hexdigest())
              for c in ChunkIter.from_config(cfg, data, 0)]
    assert chunks == [tuple(x) for x in g["chunks"]]


def test_chunk_empty(gpu_ctx):
    """rabin.rs:360-376: empty input -> no chunk, whatever the size hint."""
    from rustic_core_amd import ChunkIter, ConfigFile
    cfg = ConfigFile.new(2, oracle.DEFAULT_POLY)
    assert list(ChunkIter.from_config(cfg, b"", 0)) == []
    assert list(ChunkIter.from_config(cfg, b"", 100)) == []


def test_c1_stdrng_256mib_file(gpu_ctx, tmp_path):
    """C1 (BASELINE.json configs[0]): one 256 MiB file of
    StdRng::seed_from_u64(0x256) bytes, read by ChunkIter.from_config as
    FileArchiver::backup_reader does (file_archiver.rs:144-160) -- through
    rcdc_stream_feed -- vs the oracle on the same bytes."""
    from rustic_core_amd import ChunkIter, ConfigFile
    n = 256 * MiB
    data = oracle.stdrng_bytes(0x256, n)
    path = tmp_path / "c1.bin"
    path.write_bytes(data.tobytes())
    cfg = ConfigFile.new(2, oracle.DEFAULT_POLY)
    with open(path, "rb") as f:
        lens = [len(c) for c in ChunkIter.from_config(cfg, f, n)]
    exp = oracle.chunk_cuts(data)
    assert np.array_equal(np.cumsum(lens, dtype=np.uint64), exp)
    assert sum(lens) == n


def test_chunk_zeros(gpu_ctx):
    """rabin.rs:378-385: zeros -> first chunk is exactly MIN_SIZE."""
    from rustic_core_amd import ChunkIter, ConfigFile
    cfg = ConfigFile.new(2, oracle.DEFAULT_POLY)
    it = ChunkIter.from_config(cfg, bytes(3 * MiB + 12345), 2 ** 63)
    first = next(it)
    assert len(first) == 512 * KiB
    rest = [len(c) for c in it]
    assert rest == [512 * KiB] * 5 + [12345]


# ---------------------------------------------------------------- C2 workload
def test_c2_random_1mib_buffers(gpu_ctx):
    """Config #2 sample: 1 MiB random buffers (StdRng seed 1000+i), every cut diffed."""
    bufs = [oracle.stdrng_bytes(1000 + i, MiB) for i in range(256)]
    got = _device_cuts(gpu_ctx, bufs)
    for i, b in enumerate(bufs):
        assert np.array_equal(got[i], oracle.chunk_cuts(b)), i


def test_batch_host_api(gpu_ctx):
    bufs = [oracle.stdrng_bytes(7 + i, n) for i, n in
            enumerate([0, 1, 63, 4096, 512 * KiB, 512 * KiB + 64, 512 * KiB + 65, 3 * MiB + 7])]
    got = gpu_ctx.chunk_batch(bufs)
    for i, b in enumerate(bufs):
        assert np.array_equal(got[i], oracle.chunk_cuts(b)), i


# ---------------------------------------------------------------- edge sizes
@pytest.mark.parametrize("n", [0, 1, 64, 4095, 512 * KiB - 1, 512 * KiB, 512 * KiB + 1,
                               512 * KiB + 63, 512 * KiB + 64, 512 * KiB + 65,
                               512 * KiB + 200, MiB, 8 * MiB, 8 * MiB + 1, 17 * MiB + 3])
def test_edge_lengths(gpu_ctx, n):
    b = oracle.stdrng_bytes(99, n)
    got = _device_cuts(gpu_ctx, [b])[0]
    assert np.array_equal(got, oracle.chunk_cuts(b))


def test_unaligned_offsets(gpu_ctx):
    bufs = [oracle.stdrng_bytes(300 + i, MiB + 17 * i) for i in range(6)]
    offsets, o = [], 0
    for b in bufs:
        o += 1 + 37 * len(offsets)
        offsets.append(o)
        o += len(b)
    got = _device_cuts(gpu_ctx, bufs, offsets=offsets)
    for i, b in enumerate(bufs):
        assert np.array_equal(got[i], oracle.chunk_cuts(b)), i


# ---------------------------------------------------------------- small params
def _mixed(seed, n, zero_frac=0.5):
    rng = np.random.default_rng(seed)
    out = np.empty(n, dtype=np.uint8)
    i = 0
    while i < n:
        k = int(rng.integers(1, 40000))
        if rng.random() < zero_frac:
            out[i:i + k] = 0
        else:
            out[i:i + k] = rng.integers(0, 256, size=len(out[i:i + k]), dtype=np.uint8)
        i += k
    return out


@pytest.mark.parametrize("params", [(4096, 8192, 16384), (4096, 4096, 4096),
                                    (4096, 16384, 65536), (8192, 65536, 1 << 20),
                                    (4096, 4096, 1 << 16), (5000, 8192, 12000)])
@pytest.mark.parametrize("kind", ["random", "zeros", "mixed", "lowent"])
def test_small_params(params, kind):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mn, avg, mx = params
    ctx = _ctx(mn, avg, mx)
    n = 3 * MiB + 1234
    if kind == "random":
        b = oracle.stdrng_bytes(5, n)
    elif kind == "zeros":
        b = np.zeros(n, np.uint8)
    elif kind == "mixed":
        b = _mixed(11, n)
    else:
        b = np.random.default_rng(3).integers(0, 2, size=n, dtype=np.uint8)
    got = _device_cuts(ctx, [b, b[:n // 3], b[7:]])
    for g, x in zip(got, [b, b[:n // 3], b[7:]]):
        exp = oracle.chunk_cuts(x, min_size=mn, avg=avg, max_size=mx)
        assert np.array_equal(g, exp)


def test_other_polynomial():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # deg 53 (other taps), 40, 56 and the low degrees 9..33 whose top byte
    # straddles the two state words (generic runtime-shift instantiation)
    for poly in (0x3DA3358B4DC173 ^ (1 << 20), (1 << 40) | 0x1B, (1 << 56) | 0x95,
                 (1 << 9) | 0x11, (1 << 20) | 0x9, (1 << 31) | 0x9, (1 << 32) | 0x8D,
                 (1 << 33) | 0x53):
        ctx = _ctx(4096, 8192, 65536, poly)
        b = oracle.stdrng_bytes(17, 2 * MiB)
        got = _device_cuts(ctx, [b])[0]
        exp = oracle.chunk_cuts(b, poly=poly, min_size=4096, avg=8192, max_size=65536)
        assert np.array_equal(got, exp), hex(poly)


# ---------------------------------------------------------------- min-zone (V1)
def test_min_zone_v1_semantics():
    """Inputs crafted so that a min-zone position hits under V1 only or A only."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tests.zone_craft import craft_zone_cases
    mn, avg, mx = 4096, 1 << 16, 1 << 20
    ctx = _ctx(mn, avg, mx)
    cases = craft_zone_cases(mn, avg, count=24)
    bufs = [c for c, _ in cases]
    got = _device_cuts(ctx, bufs)
    n_diff = 0
    for g, b in zip(got, bufs):
        v1 = oracle.chunk_cuts(b, min_size=mn, avg=avg, max_size=mx)
        a = oracle.chunk_cuts(b, min_size=mn, avg=avg, max_size=mx, prefill64=True)
        n_diff += not np.array_equal(v1, a)
        assert np.array_equal(g, v1)
    assert n_diff >= len(bufs) // 2


# ---------------------------------------------------------------- streaming
def test_stream_split_invariance(gpu_ctx):
    """Cuts do not depend on how the file is split into reads (rabin.rs:162-181)."""
    from rustic_core_amd.chunker import _Stream
    b = _mixed(21, 40 * MiB, 0.3)
    exp = oracle.chunk_cuts(b)
    rng = np.random.default_rng(5)
    for trial in range(3):
        st = _Stream(gpu_ctx)
        cuts, i = [], 0
        while i < b.size:
            k = int(rng.integers(1, 24 * MiB))
            piece = b[i:i + k].tobytes()
            i += len(piece)
            cuts.extend(st.feed(piece, i >= b.size).tolist())
        if b.size == 0:
            cuts.extend(st.feed(b"", True).tolist())
        st.close()
        assert np.array_equal(np.array(cuts, np.uint64), exp), trial


def test_chunkiter_large_mixed(gpu_ctx):
    from rustic_core_amd import ChunkIter, ConfigFile
    b = _mixed(8, 70 * MiB, 0.5)
    cfg = ConfigFile.new(2, oracle.DEFAULT_POLY)
    lens = [len(c) for c in ChunkIter.from_config(cfg, b.tobytes(), 0)]
    assert np.array_equal(np.cumsum(lens, dtype=np.uint64), oracle.chunk_cuts(b))


# ------------------------------------------------------- long streams: pieces
def _phase_zeros(n, phase, seed):
    """random prefix of `phase` bytes, then zeros: the speculative chains from
    piece starts (multiples of min) run out of phase with the true chain."""
    rng = np.random.default_rng(seed)
    a = np.zeros(n, np.uint8)
    a[:phase] = rng.integers(0, 256, phase, dtype=np.uint8)
    return a


@pytest.mark.parametrize("kind", ["random", "zeros", "mixed", "phase_zeros", "lowent"])
def test_long_stream_pieces_small_params(kind, monkeypatch):
    """Speculative pieces + stitch (rcdc_resolve.hip) on long streams with
    many pieces: bit-exact whatever the merge behaviour."""
    mn, avg, mx = 4096, 16384, 65536
    monkeypatch.setenv("RCDC_PIECE_BYTES", str(16 * mn))
    rng = np.random.default_rng(11)
    n = 6 * MiB + 777
    if kind == "random":
        data = rng.integers(0, 256, n, dtype=np.uint8)
    elif kind == "zeros":
        data = np.zeros(n, np.uint8)
    elif kind == "mixed":
        data = _mixed(5, n)
    elif kind == "phase_zeros":
        data = _phase_zeros(n, 1234, 3)
    else:
        data = rng.integers(0, 3, n, dtype=np.uint8)
    ctx = _ctx(mn, avg, mx)
    got = _device_cuts(ctx, [data, data[: n // 3], data[5:]])
    for g, b in zip(got, [data, data[: n // 3], data[5:]]):
        assert np.array_equal(g, oracle.chunk_cuts(b, oracle.DEFAULT_POLY, mn, avg, mx))


@pytest.mark.parametrize("kind", ["random", "zeros", "phase_zeros", "mixed"])
def test_long_stream_default_params(gpu_ctx, kind, monkeypatch):
    """Default parameters, 160 MiB streams: the automatic piece size (and a
    forced small one) give the oracle's cuts."""
    n = 160 * MiB + 4097
    if kind == "random":
        data = oracle.stdrng_bytes(77, n)
    elif kind == "zeros":
        data = np.zeros(n, np.uint8)
    elif kind == "phase_zeros":
        data = _phase_zeros(n, 3 * MiB + 99, 4)
    else:
        data = _mixed(9, n)
    want = oracle.chunk_cuts(data)
    assert np.array_equal(_device_cuts(gpu_ctx, [data])[0], want)
    monkeypatch.setenv("RCDC_PIECE_BYTES", str(8 * MiB))
    assert np.array_equal(_device_cuts(gpu_ctx, [data])[0], want)


def test_pipelined_runs(gpu_ctx):
    """rcdc_plan_set_pipeline: resolve k on the plan's stream overlaps scan
    k + 1 (ping-pong summaries); alternating arenas must give each run's own
    cuts, and the fused hash must follow the last run."""
    import hashlib
    torch = _torch()
    from rustic_core_amd.device import DevicePlan, pack_offsets
    lens = [MiB] * 96 + [3 * MiB + 17, 524288 + 65, 100]
    offs, arena_len = pack_offsets(lens)
    hosts = []
    for a in range(2):
        h = np.zeros(arena_len, dtype=np.uint8)
        for i, (o, n) in enumerate(zip(offs, lens)):
            h[int(o):int(o) + n] = oracle.stdrng_bytes(7000 + 1000 * a + i, n)
        hosts.append(h)
    devs = [torch.from_numpy(h).to("cuda:0") for h in hosts]
    exp = [[oracle.chunk_cuts(h[int(o):int(o) + n]) for o, n in zip(offs, lens)] for h in hosts]
    plan = DevicePlan(gpu_ctx, offs, lens, arena_len)
    plan.set_pipeline(True)
    for k in range(7):
        plan.run(devs[k % 2].data_ptr())
    got = plan.results()  # last run: arena 0
    assert all(np.array_equal(g, e) for g, e in zip(got, exp[0]))
    for k in range(3):
        plan.run(devs[(k + 1) % 2].data_ptr())
    plan.hash(devs[1].data_ptr())
    got = plan.results()
    assert all(np.array_equal(g, e) for g, e in zip(got, exp[1]))
    digs = plan.digests()
    h = hosts[1]
    for i in (0, 96, 97):
        o, prev = int(offs[i]), 0
        for j, c in enumerate(got[i]):
            assert bytes(digs[i][j]) == hashlib.sha256(h[o + prev:o + int(c)].tobytes()).digest()
            prev = int(c)
    plan.set_pipeline(False)
    plan.run(devs[0].data_ptr())
    assert all(np.array_equal(g, e) for g, e in zip(plan.results(), exp[0]))
    plan.close()
