"""The native ingest engine through its C ABI (rcdc_ingest_*, ctypes): files
-> pack files + pack ids in host memory, checked against the oracle and
hashlib end to end.

Reference: FileArchiver::backup_reader (archiver/file_archiver.rs:144-160)
chunks each file, hashes each chunk (crypto/hasher.rs:17-19), skips ids the
index or the packer has (blob/packer.rs:304-315), compresses + seals +
verifies each new blob (backend/decrypt.rs:478-529), packs them by PackSizer
(packer.rs:65-200, 659-671) with a sealed header (:693-735), and names each
pack by the SHA-256 of its bytes (:826-836).

Every check is independent of the engine: cuts against oracle/cdc_ref, chunk
ids and pack ids against hashlib, pack headers opened and parsed by the
oracle's AES/Poly1305 + header restatement, every blob opened, decoded by
libzstd and hashed back to its id, and the dedup decisions against a plain
Python replay of Packer::add in file order.
"""
import hashlib
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEY = bytes(range(7, 71))


def _files():
    from oracle import oracle
    rng = np.random.default_rng(55)
    fs = []
    fs.append(rng.integers(0, 256, 3 << 20, dtype=np.uint8))          # random
    fs.append(np.zeros(10 << 20, np.uint8))                           # zeros: min chunks, dups
    fs.append(np.zeros(0, np.uint8))                                  # empty
    fs.append(rng.integers(0, 256, 100, dtype=np.uint8))              # tiny
    m = np.zeros(30 << 20, np.uint8)                                  # mixed
    i = 0
    while i < m.size:
        k = int(rng.integers(64 << 10, 4 << 20))
        if rng.random() < 0.5:
            m[i:i + k] = rng.integers(0, 256, len(m[i:i + k]), dtype=np.uint8)
        i += k
    fs.append(m)
    fs.append(oracle.stdrng_bytes(23, 32 << 20))                      # the snapshot's bytes
    fs.append(fs[0].copy())                                           # a duplicate file
    fs.append(np.frombuffer(b"a,b,c\n1,2,3\n" * 400000, np.uint8).copy())  # text (compressible)
    fs.append(rng.integers(0, 256, (20 << 20) + 3, dtype=np.uint8))
    return fs


def _replay(files, cuts_per_file, index_ids):
    """Packer::add in file order: the first occurrence of an id not indexed."""
    seen = set(index_ids)
    new = []
    for data, cuts in zip(files, cuts_per_file):
        prev = 0
        for c in cuts:
            d = hashlib.sha256(data[prev:int(c)].tobytes()).digest()
            if d not in seen:
                seen.add(d)
                new.append(d)
            prev = int(c)
    return new


def _run(gpu_ctx, files, level=0, via_path=None, threads=1, index_ids=(), **cfg):
    from rustic_core_amd.native_ingest import NativeIngest
    ing = NativeIngest(gpu_ctx, KEY, level=level, **cfg)
    try:
        if index_ids:
            ing.add_index(np.frombuffer(b"".join(index_ids), np.uint8))
        if threads == 1:
            for i, f in enumerate(files):
                if via_path:
                    ing.add_file(i, via_path[i])
                else:
                    ing.add(i, f)
        else:
            nxt = [0]
            lk = threading.Lock()

            def worker():
                while True:
                    with lk:
                        i = nxt[0]
                        nxt[0] += 1
                    if i >= len(files):
                        return
                    ing.add(i, files[i])
            ts = [threading.Thread(target=worker) for _ in range(threads)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        stats = ing.finish()
        return ing, stats
    except BaseException:
        ing.close()
        raise


def _check_all(files, ing, stats, level, index_ids=(), params=None):
    """params: (poly, min, avg, max) of the engine's context (default: rustic's)."""
    from oracle import oracle, zstd_ref
    assert stats["files"] == len(files) == len(ing.files)
    want_cuts = [oracle.chunk_cuts(f, *params) if params else oracle.chunk_cuts(f) for f in files]
    for i, f in enumerate(files):
        cuts, ids, nnew, ln = ing.files[i]
        assert ln == f.size
        assert np.array_equal(cuts, want_cuts[i]), i
        prev = 0
        for j, c in enumerate(cuts):
            assert bytes(ids[j]) == hashlib.sha256(f[prev:int(c)].tobytes()).digest(), (i, j)
            prev = int(c)
    new = _replay(files, want_cuts, index_ids)
    assert stats["new_blobs"] == len(new)
    assert sum(v[2] for v in ing.files.values()) == len(new)
    # packs: ids, headers, every blob back to its id; the blobs in packer order
    by_id = {}
    for i, f in enumerate(files):
        prev = 0
        for c in want_cuts[i]:
            by_id.setdefault(hashlib.sha256(f[prev:int(c)].tobytes()).digest(), f[prev:int(c)])
            prev = int(c)
    packed = []
    assert [p["seq"] for p in ing.packs] == list(range(len(ing.packs)))
    assert stats["packs"] == len(ing.packs)
    for p in ing.packs:
        data = p["data"]
        assert len(data) == p["size"]
        assert hashlib.sha256(data).digest() == p["id"]
        parsed = oracle.parse_pack(KEY, data)
        assert len(parsed) == len(p["blobs"])
        end = 0
        for (tpe, off, ln, ulen, bid), (id_, boff, blen, bulen, btype) in zip(parsed, p["blobs"]):
            assert (tpe == 0 or tpe == 2) and btype == 0
            assert off == boff and ln == blen and bytes(bid) == id_ and ulen == bulen
            plain = oracle.open_(KEY, data[off:off + ln])
            raw = zstd_ref.decompress(plain) if level is not None else plain
            assert hashlib.sha256(raw).digest() == id_
            assert (ulen == len(raw)) if level is not None else ulen == 0
            end = off + ln
            packed.append(id_)
        assert end + p["header_len"] + 4 == p["size"]
    assert packed == new  # every new blob exactly once, in Packer::add order


def test_native_ingest_end_to_end(gpu_ctx):
    """Several batches (40 MiB slots), small packs (4 MiB: packs close across
    batches, the open pack carried), both id paths (long_chunk 1 MiB), zstd
    level 3 and extra_verify on."""
    files = _files()
    ing, stats = _run(gpu_ctx, files, batch_bytes=40 << 20, pack_size=4 << 20,
                      pack_grow_factor=0, long_chunk=1 << 20, depth=3)
    try:
        assert stats["batches"] >= 3
        _check_all(files, ing, stats, 0)
    finally:
        ing.close()


def test_native_ingest_stored_blobs_and_index(gpu_ctx):
    """A version-1 repository (no compression): blobs stored sealed; ids the
    index already has are skipped (Indexer::has)."""
    from oracle import oracle
    files = _files()[:6]
    cuts = oracle.chunk_cuts(files[5])
    idx = [hashlib.sha256(files[5][int(a):int(b)].tobytes()).digest()
           for a, b in zip(np.concatenate([[0], cuts[:-1]]), cuts)][::2]
    ing, stats = _run(gpu_ctx, files, level=None, index_ids=idx, batch_bytes=48 << 20,
                      pack_size=8 << 20, depth=2, long_chunk=4 << 20)
    try:
        _check_all(files, ing, stats, None, index_ids=idx)
    finally:
        ing.close()


def test_native_ingest_files_from_disk_threads(gpu_ctx, tmp_path):
    """Files read from disk straight into the engine's page-locked slots
    (reserve / readinto / commit), and concurrent adders (archiver.rs:195)."""
    files = _files()
    paths = []
    for i, f in enumerate(files):
        p = str(tmp_path / f"f{i}")
        f.tofile(p)
        paths.append(p)
    ing, stats = _run(gpu_ctx, files, via_path=paths, batch_bytes=40 << 20,
                      pack_size=16 << 20, depth=4)
    try:
        _check_all(files, ing, stats, 0)
    finally:
        ing.close()
    ing, stats = _run(gpu_ctx, files, threads=4, batch_bytes=40 << 20, depth=4)
    try:
        # with 4 adders the file order in the slots is not the list order:
        # cuts and ids per file, and the pack/id checks, still hold
        from oracle import oracle
        for i, f in enumerate(files):
            assert np.array_equal(ing.files[i][0], oracle.chunk_cuts(f))
        for p in ing.packs:
            assert hashlib.sha256(p["data"]).digest() == p["id"]
        distinct = set()
        for i, f in enumerate(files):
            prev = 0
            for c in ing.files[i][0]:
                distinct.add(hashlib.sha256(f[prev:int(c)].tobytes()).digest())
                prev = int(c)
        assert stats["new_blobs"] == len(distinct) == sum(len(p["blobs"]) for p in ing.packs)
    finally:
        ing.close()


def test_native_ingest_rejects(gpu_ctx):
    import ctypes

    from oracle import oracle
    from rustic_core_amd import _lib
    from rustic_core_amd.errors import RusticError
    from rustic_core_amd.native_ingest import NativeIngest
    ing = NativeIngest(gpu_ctx, KEY, batch_bytes=8 << 20, depth=2)
    try:
        buf, t = ctypes.c_void_p(), ctypes.c_uint64()
        # one reservation is at most a slot; a larger file goes in as a stream
        assert _lib.lib().rcdc_ingest_reserve(ing._h, 9 << 20, ctypes.byref(buf),
                                              ctypes.byref(t)) == 1  # Unsupported
        big = np.random.default_rng(5).integers(0, 256, 9 << 20, dtype=np.uint8)
        ing.add(0, big)  # rcdc_ingest_add: pieces of a stream
        ing.add(1, np.ones(1000, np.uint8))
        h = ing.stream_open(2)
        with pytest.raises(RusticError):  # a piece larger than a slot
            ing.stream_reserve(h, 9 << 20)
        mv, tk = ing.stream_reserve(h, 4096)
        with pytest.raises(RusticError):  # a piece still reserved
            ing.stream_close(h)
        with pytest.raises(RusticError):  # open streams block finish
            ing.finish()
        mv[:] = b"z" * 4096
        ing.commit(tk, 4096)
        ing.stream_close(h)
        with pytest.raises(RusticError):  # the handle is gone
            ing.stream_reserve(h, 10)
        stats = ing.finish()
        assert stats["files"] == 3
        assert np.array_equal(ing.files[0][0], oracle.chunk_cuts(big))
        assert list(ing.files[2][0]) == [4096]
        with pytest.raises(RusticError):  # after finish
            ing.add(3, b"x")
    finally:
        ing.close()
