"""The native ingest engine with inputs of any length (rcdc_ingest_stream_*),
cancelled reservations, MAX_AGE pack saves, failure-safe creation and one
dedup set shared by two engines -- through the C ABI (ctypes), checked
against the oracle and hashlib.

Reference: ChunkIter::from_config(&config, reader, size_hint)
(chunker.rs:22-47) chunks any `Read`, size_hint only a capacity hint; its
iterator (rabin.rs:110-191) reads until Ok(0).  backup --stdin feeds a
child's stdout or stdin (commands/backup.rs:336-346).  A file whose read
fails is logged and skipped (archiver.rs:197-203) -- the chunks it yielded
before the error were already handed to Packer::add
(file_archiver.rs:144-160).  The packer saves a pack older than MAX_AGE
(packer.rs:63, 668-670).  One Packer per backup stores each blob once
(archiver.rs:195, packer.rs:304-315).
"""
import hashlib
import io
import threading
import time

import numpy as np
import pytest

from tests.test_gpu_native_ingest import KEY, _check_all, _replay

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _mixed(n, seed):
    rng = np.random.default_rng(seed)
    m = np.zeros(n, np.uint8)
    i = 0
    while i < n:
        k = int(rng.integers(64 << 10, 4 << 20))
        if rng.random() < 0.5:
            m[i:i + k] = rng.integers(0, 256, len(m[i:i + k]), dtype=np.uint8)
        i += k
    return m


class ChoppyReader:
    """A Read of unknown length: short reads of random sizes (a pipe)."""

    def __init__(self, data, seed):
        self.data, self.pos = data, 0
        self.rng = np.random.default_rng(seed)

    def readinto(self, mv):
        k = min(len(mv), int(self.rng.integers(1, 3 * MiB)), len(self.data) - self.pos)
        if k <= 0:
            return 0
        mv[:k] = self.data[self.pos:self.pos + k].tobytes()
        self.pos += k
        return k


class FailingReader(ChoppyReader):
    def __init__(self, data, seed, fail_at):
        super().__init__(data, seed)
        self.fail_at = fail_at

    def readinto(self, mv):
        if self.pos >= self.fail_at:
            raise OSError("read failed")
        mv = mv[:max(self.fail_at - self.pos, 0)]
        return super().readinto(mv)


def _ingest(gpu_ctx, **cfg):
    from rustic_core_amd.native_ingest import NativeIngest
    return NativeIngest(gpu_ctx, KEY, level=0, **cfg)


def test_stream_files_larger_than_a_batch(gpu_ctx):
    """batch_bytes = 40 MiB: a 300 MiB file (rcdc_ingest_add: a stream of
    quarter-batch pieces), a 5 x batch file fed in 7 MiB pieces, a stream of
    unknown length with short reads, small files around them.  Every cut vs
    the oracle, every id vs hashlib, every pack opened by the oracle, the
    dedup order replayed (files fed one after another, so Packer::add order
    is the list order)."""
    rng = np.random.default_rng(61)
    files = [
        rng.integers(0, 256, 3 * MiB, dtype=np.uint8),
        _mixed(300 * MiB, 62),
        np.frombuffer(b"x,y\n" * 100000, np.uint8).copy(),
        _mixed(200 * MiB + 12345, 63),
        np.zeros(5 * MiB, np.uint8),
        _mixed(90 * MiB + 7, 64),
        rng.integers(0, 256, 1000, dtype=np.uint8),
    ]
    files.append(files[3][:50 * MiB].copy())  # a prefix of the streamed file: shared chunks
    ing = _ingest(gpu_ctx, batch_bytes=40 * MiB, pack_size=8 * MiB, pack_grow_factor=0,
                  long_chunk=1 * MiB, depth=3)
    try:
        for i, f in enumerate(files):
            if i == 3:
                n = ing.add_stream(i, io.BytesIO(f.tobytes()), piece=7 * MiB, size_hint=f.size)
                assert n == f.size
            elif i == 5:
                assert ing.add_stream(i, ChoppyReader(f, 65), piece=5 * MiB) == f.size
            else:
                ing.add(i, f)
        stats = ing.finish()
        assert stats["batches"] >= 15
        _check_all(files, ing, stats, 0)
    finally:
        ing.close()


def test_streams_interleaved_threads(gpu_ctx):
    """Four readers stream four files at once in 3 MiB pieces: pieces of a
    stream interleave with the others' in every slot (gathered into the
    assembly region), and each batch carries every stream's open chunk."""
    files = [_mixed(70 * MiB + k * 333, 70 + k) for k in range(4)]
    files[2][:20 * MiB] = files[0][:20 * MiB]  # chunks found by two streams
    ing = _ingest(gpu_ctx, batch_bytes=24 * MiB, pack_size=4 * MiB, pack_grow_factor=0,
                  depth=3, max_streams=4)
    try:
        errs = []

        def run(i):
            try:
                ing.add_stream(i, ChoppyReader(files[i], 80 + i), piece=3 * MiB)
            except BaseException as e:  # pragma: no cover
                errs.append(e)
        ts = [threading.Thread(target=run, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs
        stats = ing.finish()
        from oracle import oracle
        distinct = set()
        for i, f in enumerate(files):
            cuts, ids, _, ln = ing.files[i]
            assert ln == f.size
            assert np.array_equal(cuts, oracle.chunk_cuts(f)), i
            prev = 0
            for j, c in enumerate(cuts):
                d = hashlib.sha256(f[prev:int(c)].tobytes()).digest()
                assert bytes(ids[j]) == d
                distinct.add(d)
                prev = int(c)
        packed = [b[0] for p in ing.packs for b in p["blobs"]]
        assert len(packed) == len(set(packed)) == len(distinct) == stats["new_blobs"]
        for p in ing.packs:
            assert hashlib.sha256(p["data"]).digest() == p["id"]
            assert oracle.parse_pack(KEY, p["data"])
    finally:
        ing.close()


def test_cancel_and_abort(gpu_ctx):
    """A cancelled reservation beside committed files: no result for it and
    finish returns.  A stream whose read fails mid-way is aborted: no file
    result, and the chunks it completed before the failure are packed
    (Packer::add ran for them in the reference), the open one is dropped."""
    from oracle import oracle
    rng = np.random.default_rng(90)
    a = rng.integers(0, 256, 2 * MiB, dtype=np.uint8)
    b = _mixed(30 * MiB, 91)
    bad = _mixed(60 * MiB, 92)
    fail_at = 37 * MiB + 11
    fed = 36 * MiB  # the 4 MiB pieces read in full before the failing one
    ing = _ingest(gpu_ctx, batch_bytes=16 * MiB, pack_size=4 * MiB, pack_grow_factor=0, depth=2)
    try:
        ing.add(0, a)
        import ctypes
        from rustic_core_amd import _lib
        buf, t = ctypes.c_void_p(), ctypes.c_uint64()
        assert _lib.lib().rcdc_ingest_reserve(ing._h, 5 * MiB, ctypes.byref(buf),
                                              ctypes.byref(t)) == 0
        ing.cancel(t.value)
        with pytest.raises(Exception):  # the ticket is spent
            ing.commit(t.value, 0, 99)
        with pytest.raises(OSError):
            ing.add_stream(2, FailingReader(bad, 93, fail_at), piece=4 * MiB)
        ing.add(1, b)
        stats = ing.finish()
        assert sorted(ing.files) == [0, 1] and stats["files"] == 2
        for i, f in ((0, a), (1, b)):
            assert np.array_equal(ing.files[i][0], oracle.chunk_cuts(f))
        # the aborted stream: every chunk final before the failure is packed
        pre = oracle.chunk_cuts(bad[:fed])
        done = []
        prev = 0
        for c in pre[:-1]:
            done.append(hashlib.sha256(bad[prev:int(c)].tobytes()).digest())
            prev = int(c)
        assert len(done) >= 20
        packed = {b_[0] for p in ing.packs for b_ in p["blobs"]}
        assert set(done) <= packed
        tail = hashlib.sha256(bad[prev:fed].tobytes()).digest()
        assert tail not in packed
        want = set(_replay([a, b], [oracle.chunk_cuts(a), oracle.chunk_cuts(b)], ())) | set(done)
        assert packed == want and stats["new_blobs"] == len(want)
    finally:
        ing.close()


def test_pack_max_age_trickle(gpu_ctx):
    """A trickle of small files: the open slot is submitted after
    slot_max_age_ms and the open pack saved after pack_max_age_ms, before
    finish (MAX_AGE, packer.rs:668-670)."""
    ing = _ingest(gpu_ctx, batch_bytes=16 * MiB, pack_size=32 * MiB, depth=2,
                  pack_max_age_ms=400, slot_max_age_ms=100)
    try:
        rng = np.random.default_rng(95)
        f0 = rng.integers(0, 256, 200000, dtype=np.uint8)
        ing.add(0, f0)
        t0 = time.time()
        while time.time() - t0 < 10 and not ing.packs:
            time.sleep(0.05)
        assert len(ing.packs) == 1, "the aged pack was not saved before finish"
        assert ing.files[0][3] == f0.size
        f1 = rng.integers(0, 256, 300000, dtype=np.uint8)
        ing.add(1, f1)
        stats = ing.finish()
        _check_all([f0, f1], ing, stats, 0)
        assert len(ing.packs) == 2
    finally:
        ing.close()


def test_pack_buffer_regrow(gpu_ctx):
    """Packs larger than the device pack buffer (max_streams 1: ~113 MiB at
    40 MiB batches) with earlier packs' copies back still queued: the
    regrow waits for them, every pack decodes to its blobs."""
    files = [np.random.default_rng(100 + k).integers(0, 256, 36 * MiB, dtype=np.uint8)
             for k in range(8)]
    ing = _ingest(gpu_ctx, batch_bytes=40 * MiB, pack_size=130 * MiB, pack_grow_factor=0,
                  depth=3, max_streams=1)
    try:
        for i, f in enumerate(files):
            ing.add(i, f)
        stats = ing.finish()
        assert max(p["size"] for p in ing.packs) > 120 * MiB
        _check_all(files, ing, stats, 0)
    finally:
        ing.close()


def test_create_failures_free_everything(gpu_ctx, monkeypatch):
    """A failure at any allocation of rcdc_ingest_create leaves nothing
    allocated (rcdc_ingest_mem_live back to zero); a good create holds
    exactly rcdc_ingest_footprint."""
    from rustic_core_amd.errors import RusticError
    from rustic_core_amd.native_ingest import NativeIngest, footprint, mem_live
    cfg = dict(batch_bytes=16 * MiB, depth=2, in_slots=2, out_slots=2, max_streams=2)
    assert mem_live() == (0, 0)
    for k in (1, 2, 3, 5, 6, 8, 11, 14, 17):
        monkeypatch.setenv("RCDC_INGEST_FAIL_ALLOC", str(k))
        with pytest.raises(RusticError):
            NativeIngest(gpu_ctx, KEY, **cfg)
        assert mem_live() == (0, 0), k
    monkeypatch.delenv("RCDC_INGEST_FAIL_ALLOC")
    ing = NativeIngest(gpu_ctx, KEY, **cfg)
    try:
        assert mem_live() == footprint(gpu_ctx, **cfg)
        ing.add(0, b"hello" * 1000)
        ing.finish()
    finally:
        ing.close()
    assert mem_live() == (0, 0)


def test_two_engines_one_dedup_set(gpu_ctx):
    """Multi-device ingest: two engines (both on cuda:0 here, one per GPU on
    a node) behind a size-balancing router, sharing one dedup set.  Files
    repeat across the engines; every distinct chunk id is packed exactly once
    over both engines' packs, every cut matches the oracle, every pack opens
    and its blobs hash back to their ids."""
    from oracle import oracle, zstd_ref
    from rustic_core_amd.native_ingest import MultiIngest
    base = [_mixed(12 * MiB + k, 110 + k) for k in range(6)]
    files = []
    for k in range(6):
        files.append(base[k])
        files.append(base[(k + 3) % 6].copy())  # a copy that the router sends elsewhere
    files.append(np.concatenate([base[0][:5 * MiB], base[1][:5 * MiB]]))
    idx = [hashlib.sha256(base[5][:int(oracle.chunk_cuts(base[5])[0])].tobytes()).digest()]
    m = MultiIngest([gpu_ctx, gpu_ctx], KEY, level=0, index_ids=np.frombuffer(idx[0], np.uint8),
                    batch_bytes=24 * MiB, pack_size=4 * MiB, pack_grow_factor=0, depth=2)
    try:
        for i, f in enumerate(files):
            m.add(i, f)
        stats = m.finish()
        got = m.files
        distinct = set()
        for i, f in enumerate(files):
            cuts, ids, _, _ = got[i]
            assert np.array_equal(cuts, oracle.chunk_cuts(f)), i
            prev = 0
            for j, c in enumerate(cuts):
                d = hashlib.sha256(f[prev:int(c)].tobytes()).digest()
                assert bytes(ids[j]) == d
                distinct.add(d)
                prev = int(c)
        packed = [b[0] for p in m.packs for b in p["blobs"]]
        assert len(packed) == len(set(packed)), "a blob packed twice"
        assert set(packed) == distinct - set(idx)
        assert stats["new_blobs"] == len(packed)
        assert sum(v[2] for v in got.values()) == len(packed)
        assert all(len(e.packs) for e in m.engines), "the router fed one engine only"
        for p in m.packs:
            assert hashlib.sha256(p["data"]).digest() == p["id"]
            for (tpe, off, ln, ulen, bid) in oracle.parse_pack(KEY, p["data"]):
                raw = zstd_ref.decompress(oracle.open_(KEY, p["data"][off:off + ln]))
                assert hashlib.sha256(raw).digest() == bytes(bid)
    finally:
        m.close()


def test_stream_slots_recycled(gpu_ctx):
    """max_streams = 2: a third open stream is refused while two are open;
    streams opened after closes wait for the closed ones' carry slots (their
    last batch chunked) and go on -- eight streams through two slots, one
    thread, every result checked."""
    from oracle import oracle
    from rustic_core_amd.errors import RusticError
    files = [_mixed(9 * MiB + 1000 * k, 120 + k) for k in range(8)]
    ing = _ingest(gpu_ctx, batch_bytes=16 * MiB, pack_size=4 * MiB, pack_grow_factor=0,
                  depth=2, max_streams=2)
    try:
        a, b = ing.stream_open(100), ing.stream_open(101)
        with pytest.raises(RusticError):  # max_streams open
            ing.stream_open(102)
        ing.stream_close(a)
        ing.stream_close(b)
        for i, f in enumerate(files):
            assert ing.add_stream(i, io.BytesIO(f.tobytes()), piece=5 * MiB) == f.size
        stats = ing.finish()
        assert stats["files"] == len(files) + 2
        assert ing.files[100][0].size == 0 and ing.files[101][0].size == 0  # empty streams
        for i, f in enumerate(files):
            assert np.array_equal(ing.files[i][0], oracle.chunk_cuts(f)), i
        for p in ing.packs:
            assert hashlib.sha256(p["data"]).digest() == p["id"]
    finally:
        ing.close()


@pytest.mark.parametrize("params", [
    (0x003DA3358B4DC173, 64 << 10, 256 << 10, 1 << 20),     # small chunks: many carries
    ((1 << 40) | 0x1B, 128 << 10, 512 << 10, 4 << 20),       # another degree (40)
])
def test_streams_other_parameters(params):
    """Streams and carries with a repository's other chunker parameters
    (ConfigFile chunk_size / min / max and poly, configfile.rs): the carry
    is the open chunk (< max bytes) whatever max is.  Cuts vs the oracle with
    the same parameters, ids vs hashlib, packs opened, dedup replayed."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rustic_core_amd.chunker import Context
    poly, mn, avg, mx = params
    ctx = Context.get(poly, mn, avg, mx, device=0)
    files = [_mixed(23 * MiB + 17, 71), _mixed(9 * MiB, 72),
             np.random.default_rng(73).integers(0, 256, 5 * MiB + 3, dtype=np.uint8)]
    files.append(files[0][:7 * MiB].copy())
    ing = _ingest(ctx, batch_bytes=4 * MiB, pack_size=2 * MiB, pack_grow_factor=0,
                  long_chunk=512 << 10, depth=3, max_streams=4)
    try:
        for i, f in enumerate(files):
            if i % 2 == 0:
                assert ing.add_stream(i, ChoppyReader(f, 80 + i), piece=1 * MiB + 5) == f.size
            else:
                ing.add(i, f)
        stats = ing.finish()
        assert stats["batches"] >= 10
        _check_all(files, ing, stats, 0, params=params)
    finally:
        ing.close()


def test_add_file_that_grew(gpu_ctx, tmp_path, monkeypatch):
    """A file that grew between its size and its read: the reference reads
    to EOF (rabin.rs:110-191), so add_file drops its reservation and feeds
    the whole file as a stream; cuts, ids and packs as for the full bytes."""
    import os
    files = [_mixed(6 * MiB + 999, 91), _mixed(3 * MiB, 92)]
    paths = []
    for i, f in enumerate(files):
        p = tmp_path / f"f{i}"
        p.write_bytes(f.tobytes())
        paths.append(str(p))
    real = os.path.getsize
    monkeypatch.setattr(os.path, "getsize", lambda p: max(real(p) - 4097, 0))
    ing = _ingest(gpu_ctx, batch_bytes=8 * MiB, pack_size=4 * MiB, pack_grow_factor=0)
    try:
        for i, p in enumerate(paths):
            ing.add_file(i, p)
        stats = ing.finish()
        _check_all(files, ing, stats, 0)
    finally:
        ing.close()


def test_long_chunk_inside_the_old_carry():
    """tools/soak_ingest.py seed 24: text whose chunks are all max bytes, a
    stream whose unit ends exactly at a chunk's max, so the next batch's
    first chunk is the whole carry; it is longer than long_chunk, so its id
    is hashed on the host from the carry's bytes.  Round 6 freed those bytes
    when the carry was replaced, before the host job read them (wrong ids)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rustic_core_amd.chunker import Context
    params = ((1 << 40) | 0x1B, 64 << 10, 256 << 10, 1 << 20)
    ctx = Context.get(*params, device=0)
    text = np.frombuffer(b"id,name,value\n17,alpha,3.25\n", np.uint8)
    files = [np.resize(text, 1207054).copy(), np.resize(text, 4903720).copy(),
             np.resize(text, 9 * MiB + 77).copy(), np.resize(text, 3 * MiB).copy()]
    for rep in range(3):
        ing = _ingest(ctx, batch_bytes=2 * MiB + 256, depth=1, in_slots=3, out_slots=2,
                      max_streams=1, long_chunk=256 << 10, pack_size=4 * MiB, pack_grow_factor=0,
                      hash_threads=7)
        try:
            for i, f in enumerate(files):
                ing.add(i, f)
            stats = ing.finish()
            _check_all(files, ing, stats, 0, params=params)
        finally:
            ing.close()
